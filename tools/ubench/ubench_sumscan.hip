// ubench_sumscan — where rpt::group_sum_scan_kernel's time goes (JOBDIM shape: 1e9 rows, 7630 groups).
//   sum           : group_sum_kernel (plain store of each group's sum)
//   sum+store     : the same, the sum published by a relaxed agent-scope atomic store
//   sum+count     : plain store + one relaxed agent-scope fetch_add per workgroup on one counter
//   sum+store+cnt : atomic store + fetch_add (the product kernel's non-last workgroups)
//   product       : rpt::group_sum_scan_kernel, with its offsets checked against group_sum + group_scan
// Best of 9, HIP events. Tools only; not the product.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rpt_bloom_device.hpp"
#include "kernels/common.hpp"
#include "kernels/compaction.hpp"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

using namespace rpt;

template <bool ATOMIC_STORE, bool COUNT>
__global__ __launch_bounds__(kBlockThreads) void sum_variant(const uint32_t* __restrict__ seg_counts, uint64_t n_segs,
                                                            uint32_t* __restrict__ sums, uint32_t* __restrict__ counter) {
  __shared__ uint32_t s_part[kWavesPerBlock];
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kGroupSegs + threadIdx.x;
  uint32_t s = i < n_segs ? seg_counts[i] : 0u;
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = s_part[0] + s_part[1] + s_part[2] + s_part[3];
    if (ATOMIC_STORE) __hip_atomic_store(sums + blockIdx.x, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else sums[blockIdx.x] = t;
    if (COUNT) __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void fill_counts(uint32_t* c, uint64_t n) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) c[i] = static_cast<uint32_t>((i * 0x9e3779b97f4a7c15ULL) >> 58);  // 0..63 per segment
}

template <typename F>
double best_ms(F launch, int reps = 9) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();
  CK(hipDeviceSynchronize());
  double best = 1e30;
  for (int r = 0; r < reps; r++) {
    CK(hipEventRecord(a));
    launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    best = std::min(best, static_cast<double>(ms));
  }
  return best;
}

int main() {
  const uint64_t n_rows = 1000000000ULL;
  const uint64_t n_segs = (n_rows + kSegRows - 1) / kSegRows;
  const uint32_t n_groups = static_cast<uint32_t>((n_segs + kGroupSegs - 1) / kGroupSegs);
  uint32_t *counts, *sums, *offs, *offs2, *state, *counter;
  uint64_t *cnt, *cnt2;
  CK(hipMalloc(&counts, n_segs * 4));
  CK(hipMalloc(&sums, n_groups * 4));
  CK(hipMalloc(&offs, n_groups * 4));
  CK(hipMalloc(&offs2, n_groups * 4));
  CK(hipMalloc(&state, (n_groups + 1) * 4));
  CK(hipMalloc(&counter, 4));
  CK(hipMalloc(&cnt, 8));
  CK(hipMalloc(&cnt2, 8));
  CK(hipMemset(state, 0, (n_groups + 1) * 4));
  CK(hipMemset(counter, 0, 4));
  hipLaunchKernelGGL(fill_counts, dim3((n_segs + 255) / 256), dim3(256), 0, 0, counts, n_segs);
  printf("segments %llu, groups %u\n", (unsigned long long)n_segs, n_groups);
  const dim3 grid(n_groups), blk(kBlockThreads);
  auto line = [](const char* name, double ms) { printf("%-14s %.4f ms\n", name, ms); };
  line("sum", best_ms([&] { hipLaunchKernelGGL(group_sum_kernel, grid, blk, 0, 0, counts, n_segs, sums); }));
  line("sum+store", best_ms([&] { hipLaunchKernelGGL((sum_variant<true, false>), grid, blk, 0, 0, counts, n_segs, sums, counter); }));
  line("sum+count", best_ms([&] { hipLaunchKernelGGL((sum_variant<false, true>), grid, blk, 0, 0, counts, n_segs, sums, counter); }));
  line("sum+store+cnt", best_ms([&] { hipLaunchKernelGGL((sum_variant<true, true>), grid, blk, 0, 0, counts, n_segs, sums, counter); }));
  line("scan", best_ms([&] { hipLaunchKernelGGL(group_scan_kernel, dim3(1), dim3(1024), 0, 0, sums, n_groups, offs, cnt); }));
  line("product", best_ms([&] {
         hipLaunchKernelGGL(group_sum_scan_kernel, grid, blk, 0, 0, counts, n_segs, n_groups, state, offs2, cnt2);
       }));
  // check: the product's offsets and total against group_sum + group_scan
  hipLaunchKernelGGL(group_sum_kernel, grid, blk, 0, 0, counts, n_segs, sums);
  hipLaunchKernelGGL(group_scan_kernel, dim3(1), dim3(1024), 0, 0, sums, n_groups, offs, cnt);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> a(n_groups), b(n_groups);
  uint64_t ca = 0, cb = 0;
  CK(hipMemcpy(a.data(), offs, n_groups * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), offs2, n_groups * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&ca, cnt, 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&cb, cnt2, 8, hipMemcpyDeviceToHost));
  printf("offsets %s, total %llu vs %llu\n", a == b ? "match" : "DIFFER", (unsigned long long)ca, (unsigned long long)cb);
  return a == b && ca == cb ? 0 : 1;
}
