// ubench_small_phases — where the fused small probe's first 512-row segment spends its time.
// A timestamped restatement of rpt::probe_small_kernel's phases for one workgroup (1024 threads) and
// one segment (n = 512, int64 keys in device memory, 1 Mi-key filter): mask-table fill, key loads +
// hash, filter gathers, pass-bit stores, sel tail. Wave 0 lane 0 reads wall_clock64() (100 MHz) after
// each phase, each read after a data dependence on the phase's results. Tools only; not the product.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rpt_bloom_device.hpp"
#include "rpt_gpu.h"
#include "kernels/common.hpp"
#include "kernels/probe_direct.hpp"

#define CHECK(x)                                                        \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                         \
    }                                                                   \
  } while (0)

constexpr int kPhases = 6;

__global__ __launch_bounds__(rpt::kSmallThreads) void phases_kernel(const uint64_t* __restrict__ words, uint64_t block_mask,
                                                                    rpt::KeyArgs a, uint64_t n, uint32_t* __restrict__ out_sel,
                                                                    uint64_t* __restrict__ out_count,
                                                                    uint64_t* __restrict__ stamps, uint64_t* __restrict__ sink) {
  using namespace rpt;
  constexpr uint32_t kSegs = kSmallRows / kSegRows;
  __shared__ uint64_t s_masks[kNumMasks];
  __shared__ uint64_t s_words[kSegs * kWordsPerSeg];
  __shared__ uint32_t s_cnt[kSegs];
  uint64_t t[kPhases];
  t[0] = wall_clock64();
  fill_mask_table(s_masks);
  __syncthreads();
  t[1] = wall_clock64();
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t n_segs = static_cast<uint32_t>((n + kSegRows - 1) / kSegRows);
  uint64_t h[8];
  bool ok[8];
  uint64_t dep = 0;
  if (wave < n_segs) {
    load_hashes<kKeyI64, true>(a, static_cast<uint64_t>(wave) * kSegRows, n, lane, h, ok);
#pragma unroll
    for (int j = 0; j < 8; j++) dep ^= h[j];
  }
  asm volatile("" ::"v"(dep));
  t[2] = wall_clock64();
  bool pass[8];
  uint64_t dep2 = 0;
  if (wave < n_segs) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint64_t m = mask_of(s_masks, h[j]);
      const uint64_t w = ok[j] ? words[block_of(h[j], block_mask)] : 0ULL;
      pass[j] = ok[j] && (w & m) == m;
      dep2 += pass[j];
    }
  }
  asm volatile("" ::"v"(dep2));
  t[3] = wall_clock64();
  if (wave < n_segs) store_segment_bits<kKeyI64, true>(pass, lane, wave, s_words, s_cnt);
  __syncthreads();
  t[4] = wall_clock64();
  small_sel_tail(s_words, s_cnt, n_segs, nullptr, out_sel, out_count);
  __syncthreads();
  t[5] = wall_clock64();
  if (threadIdx.x == 0) {
    for (int p = 0; p < kPhases; p++) stamps[p] = t[p];
  }
  if (dep == 0x12345 && dep2 == 7) sink[threadIdx.x] = dep;  // keeps the dependences live
}

int main(int argc, char** argv) {
  const int log_nb = 17;  // 1 MiB filter, the size a 1 Mi-key build gets
  const uint64_t n_words = 1ULL << log_nb;
  std::vector<uint64_t> hw(n_words);
  uint64_t x = 88172645463325252ULL;
  for (auto& w : hw) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    w = x & (x >> 3);  // ~25 % bits set: almost no row passes
  }
  const double pass_frac = argc > 2 ? atof(argv[2]) : 0.0;  // > 0: that fraction of blocks all ones
  if (pass_frac > 0)
    for (uint64_t i = 0; i < n_words; i++) if ((i * 2654435761ULL % 1000) < pass_frac * 1000) hw[i] = ~0ULL;
  const uint64_t n = argc > 1 ? std::min<uint64_t>(std::max(atoll(argv[1]), 1LL), 512) : 512;  // one segment
  std::vector<int64_t> keys(n);
  for (auto& k : keys) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; k = static_cast<int64_t>(x >> 20); }
  uint64_t *d_words, *d_count, *d_stamps, *d_sink;
  int64_t* d_keys;
  uint32_t* d_sel;
  CHECK(hipMalloc(&d_words, n_words * 8));
  CHECK(hipMalloc(&d_keys, n * 8));
  CHECK(hipMalloc(&d_sel, n * 4));
  CHECK(hipMalloc(&d_count, 8));
  CHECK(hipMalloc(&d_stamps, kPhases * 8));
  CHECK(hipMalloc(&d_sink, rpt::kSmallThreads * 8));
  CHECK(hipMemcpy(d_words, hw.data(), n_words * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_keys, keys.data(), n * 8, hipMemcpyHostToDevice));
  const rpt::KeyArgs a{d_keys, nullptr, nullptr, nullptr};
  const char* names[kPhases - 1] = {"mask fill + barrier", "key loads + hash", "filter gathers", "pass-bit stores + barrier",
                                    "sel tail"};
  for (int mode = 0; mode < 2; mode++) {  // 0: synchronized launches, 1: launches queued back to back
    std::vector<std::vector<double>> d(kPhases);
    std::vector<float> ev_us;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int it = 0; it < 2000; it++) {
      CHECK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(phases_kernel, dim3(1), dim3(rpt::kSmallThreads), 0, 0, d_words, n_words - 1, a, n, d_sel, d_count,
                         d_stamps, d_sink);
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(e1, 0));
      if (mode == 0 || it % 100 == 99) {
        CHECK(hipEventSynchronize(e1));
        uint64_t st[kPhases];
        CHECK(hipMemcpy(st, d_stamps, sizeof st, hipMemcpyDeviceToHost));
        for (int p = 1; p < kPhases; p++) d[p].push_back((st[p] - st[p - 1]) * 0.01);
        d[0].push_back((st[kPhases - 1] - st[0]) * 0.01);
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        ev_us.push_back(ms * 1000.f);
      }
    }
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    std::vector<double> ev(ev_us.begin(), ev_us.end());
    uint64_t cnt = 0;
    CHECK(hipMemcpy(&cnt, d_count, 8, hipMemcpyDeviceToHost));
    printf("%s launches (n = %llu rows, %llu pass, median us): event-timed %.2f, in-kernel total %.2f\n",
           mode ? "queued" : "synchronized", (unsigned long long)n, (unsigned long long)cnt, med(ev), med(d[0]));
    for (int p = 1; p < kPhases; p++) printf("  %-26s %.2f\n", names[p - 1], med(d[p]));
  }
  // the product kernel on the same inputs, queued back to back (its duration: run under rocprofv3 --kernel-trace
  // --stats and compare with phases_kernel's)
  for (int it = 0; it < 2000; it++)
    hipLaunchKernelGGL((rpt::probe_small_kernel<rpt::kKeyI64, true>), dim3(1), dim3(rpt::kSmallThreads), 0, 0, d_words,
                       n_words - 1, a, n, static_cast<const uint32_t*>(nullptr), d_sel, d_count);
  CHECK(hipDeviceSynchronize());
  uint64_t cnt2 = 0;
  CHECK(hipMemcpy(&cnt2, d_count, 8, hipMemcpyDeviceToHost));
  printf("product probe_small_kernel: %llu pass\n", (unsigned long long)cnt2);
  return 0;
}
