// Stream-rate variants for bench.py's calibration: which read and copy kernels reach the
// box's achievable HBM rate, so the calibration librpt_gpu.so exports (rpt_stream_read / rpt_stream_copy) is a
// ceiling and not another kernel's shortfall. 8 GiB buffer (past the 256 MiB Infinity Cache), best of 7, GB/s of
// bytes moved (copy: read + write).
//   read  : grid-stride 16-B loads, U in flight per lane, plain or non-temporal, G workgroups per CU
//   copy  : the same loads stored to the other half, plain or non-temporal stores
//   copy1 : one-shot grid (every lane copies U consecutive-stride 16-B units, no grid-stride loop)
//   ./ubench_stream
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

template <int U, bool NTL>
__global__ __launch_bounds__(256) void k_read(const u64x2* __restrict__ src, uint64_t n16, uint64_t* sink) {
  u64x2 acc = {0, 0};
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    u64x2 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = NTL ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; u++) acc ^= v[u];
  }
  for (; i < n16; i += stride) acc ^= src[i];
  if ((acc[0] ^ acc[1]) == 0x123456789ULL) sink[0] = 1;
}

template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_copy(const u64x2* __restrict__ src, uint64_t n16, u64x2* __restrict__ dst) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    u64x2 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = NTL ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (NTS) __builtin_nontemporal_store(v[u], dst + i + u * stride);
      else dst[i + u * stride] = v[u];
    }
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

// one-shot: block b covers units [b * 256 * U, (b + 1) * 256 * U), lane t copies units t, t + 256, ...
template <int U, bool NTS>
__global__ __launch_bounds__(256) void k_copy1(const u64x2* __restrict__ src, uint64_t n16, u64x2* __restrict__ dst) {
  const uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x;
  u64x2 v[U];
#pragma unroll
  for (int u = 0; u < U; u++) v[u] = base + u * 256 < n16 ? src[base + u * 256] : u64x2{0, 0};
#pragma unroll
  for (int u = 0; u < U; u++)
    if (base + u * 256 < n16) {
      if (NTS) __builtin_nontemporal_store(v[u], dst + base + u * 256);
      else dst[base + u * 256] = v[u];
    }
}

template <typename F>
double best_ms(F launch, int reps = 7) {
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
    best = std::min(best, (double)ms);
  }
  return best;
}

int main() {
  const uint64_t bytes = 8ULL << 30, half = bytes / 2;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  char* buf;
  uint64_t* sink;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 8));
  CK(hipMemset(buf, 0x5a, bytes));
  const u64x2* src = reinterpret_cast<const u64x2*>(buf);
  u64x2* dst = reinterpret_cast<u64x2*>(buf + half);
  const uint64_t n_all = bytes / 16, n_half = half / 16;
  auto rd = [&](const char* name, auto kern, int g) {
    const unsigned grid = cus * g;
    const double ms = best_ms([&] { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, src, n_all, sink); });
    printf("read  %-28s G=%2d  %.3f ms  %7.0f GB/s\n", name, g, ms, bytes / ms / 1e6);
  };
  auto cp = [&](const char* name, auto kern, int g) {
    const unsigned grid = cus * g;
    const double ms = best_ms([&] { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, src, n_half, dst); });
    printf("copy  %-28s G=%2d  %.3f ms  %7.0f GB/s\n", name, g, ms, 2.0 * half / ms / 1e6);
  };
  for (int g : {4, 8, 16}) {
    rd("U4 nt", k_read<4, true>, g);
    rd("U4 plain", k_read<4, false>, g);
    rd("U8 nt", k_read<8, true>, g);
  }
  for (int g : {4, 8, 16}) {
    cp("U4 ntload ntstore", k_copy<4, true, true>, g);
    cp("U4 ntload store", k_copy<4, true, false>, g);
    cp("U4 load store", k_copy<4, false, false>, g);
    cp("U8 load store", k_copy<8, false, false>, g);
    cp("U2 load store", k_copy<2, false, false>, g);
  }
  for (int u : {1, 4}) {
    const uint64_t per_block = 256ULL * u;
    const unsigned grid = (unsigned)((n_half + per_block - 1) / per_block);
    double ms = best_ms([&] {
      if (u == 1) hipLaunchKernelGGL((k_copy1<1, false>), dim3(grid), dim3(256), 0, 0, src, n_half, dst);
      else hipLaunchKernelGGL((k_copy1<4, false>), dim3(grid), dim3(256), 0, 0, src, n_half, dst);
    });
    printf("copy1 one-shot U%d plain store          %.3f ms  %7.0f GB/s\n", u, ms, 2.0 * half / ms / 1e6);
    ms = best_ms([&] {
      if (u == 1) hipLaunchKernelGGL((k_copy1<1, true>), dim3(grid), dim3(256), 0, 0, src, n_half, dst);
      else hipLaunchKernelGGL((k_copy1<4, true>), dim3(grid), dim3(256), 0, 0, src, n_half, dst);
    });
    printf("copy1 one-shot U%d nt store             %.3f ms  %7.0f GB/s\n", u, ms, 2.0 * half / ms / 1e6);
  }
  const double ms = best_ms([&] { CK(hipMemcpyAsync(dst, src, half, hipMemcpyDeviceToDevice, 0)); });
  printf("hipMemcpyAsync D2D                       %.3f ms  %7.0f GB/s\n", ms, 2.0 * half / ms / 1e6);
  CK(hipFree(buf));
  return 0;
}
