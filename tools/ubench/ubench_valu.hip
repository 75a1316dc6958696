// ubench_valu — is the whole-filter LDS probe bound by its VALU work, and what does the key hash cost there?
// Per-instruction issue rates on gfx950 (wave64 instructions per CU per clock, 4 independent chains per lane,
// full occupancy) and the murmur64 hash alone (keys/s with no memory traffic), against the probe's 1.58 ms per
// 1e9 int64 keys (profiles/r06/bench_JOBDIM.json). Tools only; not the product.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "rpt_bloom_device.hpp"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int kIters = 4096;

// 4 independent chains per lane of one instruction kind; the sink store keeps them alive
#define CHAIN_KERNEL(NAME, ASM)                                                              \
  __global__ __launch_bounds__(256) void NAME(uint32_t* sink, uint32_t seed) {              \
    uint32_t a = seed + threadIdx.x, b = a * 3u, c = a * 5u, d = a * 7u;                     \
    const uint32_t k = seed | 1u;                                                            \
    for (int i = 0; i < kIters; i++) {                                                       \
      asm volatile(ASM : "+v"(a) : "v"(k));                                                  \
      asm volatile(ASM : "+v"(b) : "v"(k));                                                  \
      asm volatile(ASM : "+v"(c) : "v"(k));                                                  \
      asm volatile(ASM : "+v"(d) : "v"(k));                                                  \
    }                                                                                        \
    if ((a ^ b ^ c ^ d) == 0x12345u) sink[0] = a;                                            \
  }
CHAIN_KERNEL(k_add, "v_add_u32 %0, %0, %1")
CHAIN_KERNEL(k_xor, "v_xor_b32 %0, %0, %1")
CHAIN_KERNEL(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
CHAIN_KERNEL(k_mul_hi, "v_mul_hi_u32 %0, %0, %1")
CHAIN_KERNEL(k_mul_u24, "v_mul_u32_u24 %0, %0, %1")

__global__ __launch_bounds__(256) void k_mad64(uint32_t* sink, uint32_t seed) {
  uint64_t a = seed + threadIdx.x, b = a * 3u, c = a * 5u, d = a * 7u;
  const uint32_t k = seed | 1u;
  for (int i = 0; i < kIters; i++) {
    asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(a) : "v"(k) : "vcc");
    asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(b) : "v"(k) : "vcc");
    asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(c) : "v"(k) : "vcc");
    asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(d) : "v"(k) : "vcc");
  }
  if ((a ^ b ^ c ^ d) == 0x12345u) sink[0] = static_cast<uint32_t>(a);
}

// murmur64 of 8 keys per lane per iteration (the probe's per-lane batch), results folded
__global__ __launch_bounds__(256) void k_murmur(uint32_t* sink, uint32_t seed) {
  uint64_t x[8], acc = 0;
  for (int j = 0; j < 8; j++) x[j] = (static_cast<uint64_t>(blockIdx.x) << 32) + threadIdx.x * 8 + j + seed;
  for (int i = 0; i < kIters / 8; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint64_t h = rpt::murmur64(x[j]);
      acc ^= h;
      x[j] += 0x9e3779b97f4a7c15ULL;
    }
  }
  if (acc == 0x12345u) sink[0] = static_cast<uint32_t>(acc);
}

template <typename F>
double best_ms(F launch, int reps = 5) {
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
  int cus = 0, clk_khz = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
  uint32_t* sink;
  CK(hipMalloc(&sink, 4));
  const unsigned grid = cus * 32;  // 32 x 256 threads per CU: full occupancy many times over
  const double waves = static_cast<double>(grid) * 4;
  const double ghz = clk_khz / 1e6;
  printf("CUs %d, max clock %.2f GHz, grid %u x 256\n", cus, ghz, grid);
  auto rate = [&](const char* name, auto kern, double instr_per_wave) {
    const double ms = best_ms([&] { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, sink, 7u); });
    const double per_cu_clk = waves * instr_per_wave / (ms * 1e-3) / cus / (ghz * 1e9);
    printf("%-12s %.3f ms  %.3f wave64 instr / CU / clock (at %.2f GHz)\n", name, ms, per_cu_clk, ghz);
  };
  rate("v_add_u32", k_add, 4.0 * kIters);
  rate("v_xor_b32", k_xor, 4.0 * kIters);
  rate("v_mul_lo_u32", k_mul_lo, 4.0 * kIters);
  rate("v_mul_hi_u32", k_mul_hi, 4.0 * kIters);
  rate("v_mul_u32_u24", k_mul_u24, 4.0 * kIters);
  rate("v_mad_u64_u32", k_mad64, 4.0 * kIters);
  const double ms = best_ms([&] { hipLaunchKernelGGL(k_murmur, dim3(grid), dim3(256), 0, 0, sink, 7u); });
  const double keys = static_cast<double>(grid) * 256 * (kIters / 8) * 8;
  printf("murmur64     %.3f ms  %.1f Gkeys/s  -> %.3f ms per 1e9 keys\n", ms, keys / ms / 1e6, 1e9 / (keys / ms));
  return 0;
}
