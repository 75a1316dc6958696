// ubench_compact — how far the direct probes' sel tail (rpt::compact_kernel) sits above its store floor, at the
// JOB-dimension shape: 1e9 result bits, p = 0.116 (JOBDIM's pass fraction), ~1.16e8 survivors (466 MB of sel).
//   compact  : the product kernel (kernels/compaction.hpp), offsets from the product group_sum / group_scan
//   stores   : the same grid, bit reads and per-step sel regions, but each wave writes its step's region with
//              placeholder values (no LDS expansion): the floor of compact's store pattern
//   stores16 : the same regions written with 16-B stores where aligned (4-B heads and tails)
//   write4   : a contiguous 466 MB write, one 4-B store per lane, one-shot grid (the plain write rate)
//   write16  : the same with 16-B stores
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

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}

// result bits with pass probability p (threshold on a per-row hash); one word per lane
__global__ void fill_bits(uint64_t* bits, uint64_t n_words, uint64_t thresh) {
  const uint64_t w = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (w >= n_words) return;
  uint64_t v = 0;
  for (int b = 0; b < 64; b++) v |= static_cast<uint64_t>(mix64(w * 64 + b) < thresh) << b;
  bits[w] = v;
}
__global__ void seg_count(const uint64_t* bits, uint64_t n_segs, uint32_t* counts) {
  const uint64_t s = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (s >= n_segs) return;
  uint32_t c = 0;
  for (uint64_t k = 0; k < kWordsPerSeg; k++) c += __popcll(bits[s * kWordsPerSeg + k]);
  counts[s] = c;
}

// compact_kernel's prologue and grid, with each step's region filled without the LDS expansion
template <bool V16>
__global__ __launch_bounds__(kBlockThreads) void stores_kernel(const uint64_t* __restrict__ bits,
                                                              const uint32_t* __restrict__ seg_counts, uint64_t n_segs,
                                                              const uint32_t* __restrict__ group_offs,
                                                              uint32_t* __restrict__ out_sel) {
  __shared__ uint32_t s_off[kGroupSegs];
  __shared__ uint32_t s_wave[kWavesPerBlock];
  const uint64_t g0 = static_cast<uint64_t>(blockIdx.x) * kGroupSegs;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t sidx = g0 + threadIdx.x;
  const uint32_t c = sidx < n_segs ? seg_counts[sidx] : 0u;
  const uint32_t incl = wave_inclusive_sum(c);
  if (lane == 63) s_wave[wave] = incl;
  __syncthreads();
  uint32_t off = group_offs[blockIdx.x] + incl - c;
  for (uint32_t w = 0; w < wave; w++) off += s_wave[w];
  s_off[threadIdx.x] = off;
  __syncthreads();
  const uint64_t n_words = n_segs * kWordsPerSeg;
  constexpr uint32_t kSteps = kGroupSegs / 8 / kWavesPerBlock;
  uint64_t words[kSteps];
#pragma unroll
  for (uint32_t i = 0; i < kSteps; i++) {
    const uint64_t wi = (g0 + (wave + i * kWavesPerBlock) * 8) * kWordsPerSeg + lane;
    words[i] = wi < n_words ? bits[wi] : 0ULL;
  }
#pragma unroll
  for (uint32_t i = 0; i < kSteps; i++) {
    const uint32_t b = wave + i * kWavesPerBlock;
    const uint64_t seg0 = g0 + b * 8;
    if (seg0 >= n_segs) break;
    const uint32_t total = wave_sum(static_cast<uint32_t>(__popcll(words[i])));
    const uint32_t o = s_off[b * 8];
    const uint32_t step_row = static_cast<uint32_t>(seg0 * kSegRows);
    if (!V16) {
      for (uint32_t q = lane; q < total; q += 64) out_sel[o + q] = step_row + q;
    } else {
      const uint32_t head0 = (4 - (o & 3)) & 3, head = head0 < total ? head0 : total;
      if (lane < head) out_sel[o + lane] = step_row + lane;
      const uint32_t body = (total - head) & ~3u;
      u32x4* dst = reinterpret_cast<u32x4*>(out_sel + o + head);
      for (uint32_t q = lane; q < body / 4; q += 64) {
        const uint32_t r = step_row + head + 4 * q;
        dst[q] = u32x4{r, r + 1, r + 2, r + 3};
      }
      const uint32_t tail = total - head - body;
      if (lane < tail) out_sel[o + head + body + lane] = step_row + head + body + lane;
    }
  }
}

__global__ void write4(uint32_t* dst, uint64_t n) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = static_cast<uint32_t>(i);
}
__global__ void write16(u32x4* dst, uint64_t n4) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint32_t r = static_cast<uint32_t>(i * 4);
  if (i < n4) dst[i] = u32x4{r, r + 1, r + 2, r + 3};
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

int main(int argc, char** argv) {
  const uint64_t n_rows = 1000000000ULL;
  const double p = argc > 1 ? atof(argv[1]) : 0.116;
  const uint64_t n_segs = (n_rows + kSegRows - 1) / kSegRows;
  const uint64_t n_words = n_segs * kWordsPerSeg;
  const uint32_t n_groups = static_cast<uint32_t>((n_segs + kGroupSegs - 1) / kGroupSegs);
  uint64_t *bits, *count;
  uint32_t *counts, *gsum, *goff, *sel, *sel2;
  CK(hipMalloc(&bits, n_words * 8));
  CK(hipMalloc(&counts, n_segs * 4));
  CK(hipMalloc(&gsum, n_groups * 4));
  CK(hipMalloc(&goff, n_groups * 4));
  CK(hipMalloc(&count, 8));
  const uint64_t thresh = static_cast<uint64_t>(p * 18446744073709551616.0);
  hipLaunchKernelGGL(fill_bits, dim3((n_words + 255) / 256), dim3(256), 0, 0, bits, n_words, thresh);
  hipLaunchKernelGGL(seg_count, dim3((n_segs + 255) / 256), dim3(256), 0, 0, bits, n_segs, counts);
  hipLaunchKernelGGL(group_sum_kernel, dim3(n_groups), dim3(kBlockThreads), 0, 0, counts, n_segs, gsum);
  hipLaunchKernelGGL(group_scan_kernel, dim3(1), dim3(1024), 0, 0, gsum, n_groups, goff, count);
  uint64_t survivors = 0;
  CK(hipMemcpy(&survivors, count, 8, hipMemcpyDeviceToHost));
  CK(hipMalloc(&sel, (survivors + 64) * 4));
  CK(hipMalloc(&sel2, (survivors + 64) * 4));
  const double mb = (n_words * 8 + survivors * 4) / 1e6;
  printf("p=%.3f rows=%llu survivors=%llu groups=%u  bytes(bits+sel)=%.0f MB\n", p, (unsigned long long)n_rows,
         (unsigned long long)survivors, n_groups, mb);
  auto line = [&](const char* name, double ms, double mbytes) {
    printf("%-10s %.4f ms  %6.0f GB/s\n", name, ms, mbytes / ms);
  };
  double ms = best_ms([&] {
    hipLaunchKernelGGL(compact_kernel, dim3(n_groups), dim3(kBlockThreads), 0, 0, bits, counts, n_segs, goff,
                       static_cast<const uint32_t*>(nullptr), sel);
  });
  line("compact", ms, mb);
  ms = best_ms([&] {
    hipLaunchKernelGGL(stores_kernel<false>, dim3(n_groups), dim3(kBlockThreads), 0, 0, bits, counts, n_segs, goff, sel2);
  });
  line("stores", ms, mb);
  ms = best_ms([&] {
    hipLaunchKernelGGL(stores_kernel<true>, dim3(n_groups), dim3(kBlockThreads), 0, 0, bits, counts, n_segs, goff, sel2);
  });
  line("stores16", ms, mb);
  ms = best_ms([&] { hipLaunchKernelGGL(write4, dim3((survivors + 255) / 256), dim3(256), 0, 0, sel2, survivors); });
  line("write4", ms, survivors * 4 / 1e6);
  ms = best_ms([&] {
    hipLaunchKernelGGL(write16, dim3((survivors / 4 + 255) / 256), dim3(256), 0, 0, reinterpret_cast<u32x4*>(sel2),
                       survivors / 4);
  });
  line("write16", ms, survivors * 4 / 1e6);
  // sanity: compact's sel equals the bits expanded on the host (the first 2^20 survivors)
  std::vector<uint32_t> h(std::min<uint64_t>(survivors, 1u << 20));
  CK(hipMemcpy(h.data(), sel, h.size() * 4, hipMemcpyDeviceToHost));
  std::vector<uint64_t> hb(n_words);
  CK(hipMemcpy(hb.data(), bits, n_words * 8, hipMemcpyDeviceToHost));
  size_t k = 0;
  for (uint64_t w = 0; w < n_words && k < h.size(); w++)
    for (uint64_t v = hb[w]; v && k < h.size(); v &= v - 1, k++)
      if (h[k] != w * 64 + __builtin_ctzll(v)) {
        printf("compact sel wrong at %zu: %u vs %llu\n", k, h[k], (unsigned long long)(w * 64 + __builtin_ctzll(v)));
        return 1;
      }
  printf("compact sel: first %zu entries match the host expansion\n", k);
  CK(hipFree(bits));
  CK(hipFree(sel));
  CK(hipFree(sel2));
  return 0;
}
