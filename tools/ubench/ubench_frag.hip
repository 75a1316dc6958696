// Fragmented-transfer micro-benchmark (MI355X): is a tile-major -> slice-major exchange cheaper when
// the fragmentation sits on the write side (partition writes runs into per-slice arrays) or on the
// read side (slice probe reads runs out of per-tile blocks, the current layout)?
//
// A D-byte array of T x P chunks of C bytes is copied three ways:
//   copy   : dst[i] = src[i]                              (streaming floor)
//   wfrag  : read [t][p] in order, write to [p][t]        (fragmented writes, contiguous reads)
//   rfrag  : write [p][t] in order, read from [t][p]      (fragmented reads, contiguous writes)
// Output: one line per (C, P, mode) with GB/s of read + write bytes.
//   ./ubench_frag [D_bytes]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

template <typename V, int MODE>
__global__ __launch_bounds__(256) void xpose(const V* __restrict__ src, V* __restrict__ dst, uint64_t T, uint64_t P,
                                             uint64_t pieces_per_chunk, uint64_t n_pieces) {
  constexpr int kU = 4;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t g0 = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g0 < n_pieces; g0 += stride * kU) {
    V v[kU];
    uint64_t d[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const uint64_t g = g0 + u * stride;
      if (g >= n_pieces) {
        d[u] = ~0ull;
        continue;
      }
      const uint64_t chunk = g / pieces_per_chunk, piece = g % pieces_per_chunk;
      uint64_t s = chunk, dc = chunk;
      if (MODE == 1) {  // read [t][p] contiguous, write [p][t]
        const uint64_t t = chunk / P, p = chunk % P;
        dc = p * T + t;
      } else if (MODE == 2) {  // write [p][t] contiguous, read [t][p]
        const uint64_t p = chunk / T, t = chunk % T;
        s = t * P + p;
      }
      v[u] = src[s * pieces_per_chunk + piece];
      d[u] = dc * pieces_per_chunk + piece;
    }
#pragma unroll
    for (int u = 0; u < kU; u++)
      if (d[u] != ~0ull) dst[d[u]] = v[u];
  }
}

template <typename V>
static float run(int mode, const void* src, void* dst, uint64_t D, uint64_t C, uint64_t P) {
  const uint64_t T = D / (C * P);
  const uint64_t ppc = C / sizeof(V);
  const uint64_t n = T * P * ppc;
  const int grid = 256 * 16;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int rep = 0; rep < 4; rep++) {
    CK(hipEventRecord(a));
    if (mode == 0)
      hipLaunchKernelGGL((xpose<V, 0>), dim3(grid), dim3(256), 0, 0, (const V*)src, (V*)dst, T, P, ppc, n);
    else if (mode == 1)
      hipLaunchKernelGGL((xpose<V, 1>), dim3(grid), dim3(256), 0, 0, (const V*)src, (V*)dst, T, P, ppc, n);
    else
      hipLaunchKernelGGL((xpose<V, 2>), dim3(grid), dim3(256), 0, 0, (const V*)src, (V*)dst, T, P, ppc, n);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep > 0 && ms < best) best = ms;
  }
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return best;
}

int main(int argc, char** argv) {
  const uint64_t D = argc > 1 ? strtoull(argv[1], nullptr, 10) : (4ull << 30);
  void *src, *dst;
  CK(hipMalloc(&src, D));
  CK(hipMalloc(&dst, D));
  CK(hipMemset(src, 1, D));
  CK(hipMemset(dst, 0, D));
  const char* names[3] = {"copy", "wfrag", "rfrag"};
  struct Cfg {
    uint64_t C, P;
  } cfgs[] = {{4096, 128}, {1024, 128}, {512, 128}, {256, 128}, {128, 1024}, {128, 128}, {64, 1024},
              {32, 1024},  {16, 1024}, {16, 128},  {4, 1024},   {4, 128}};
  for (const Cfg& c : cfgs) {
    for (int mode = 0; mode < 3; mode++) {
      float ms = c.C >= 16 ? run<uint4>(mode, src, dst, D, c.C, c.P) : run<uint32_t>(mode, src, dst, D, c.C, c.P);
      const uint64_t T = D / (c.C * c.P);
      const double bytes = 2.0 * static_cast<double>(T * c.P * c.C);
      printf("C=%5llu B  P=%5llu  %-6s %8.3f ms  %7.1f GB/s\n", (unsigned long long)c.C, (unsigned long long)c.P,
             names[mode], ms, bytes / (ms * 1e-3) / 1e9);
      fflush(stdout);
    }
  }
  CK(hipFree(src));
  CK(hipFree(dst));
  return 0;
}
