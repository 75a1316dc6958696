// ubench_probe.hip — microbenchmarks that decide the probe design on gfx950 (developer tool).
//
//   stream      : read 1e9 int64 keys (16-B loads) and fold them (HBM stream floor)
//   hash        : stream + murmur64 + LDS mask lookup (ALU + HBM floor)
//   gather L    : the current probe core against a 2^L-word filter (L2 / MALL / HBM gather rate)
//   lds L       : the probe with the whole 2^L-word filter staged in LDS (L <= 14)
//   mallrw S    : write then read an S-byte buffer repeatedly (does an intermediate stay in MALL?)
// Prints one line per measurement: name, param, ms, Gkeys/s (or GB/s).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rpt_bloom_device.hpp"

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

using namespace rpt;
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint64_t smx(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

__global__ void gen_keys(int64_t* k, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    k[i] = (int64_t)smx(0x1234 + (i + 1) * 0x9e3779b97f4a7c15ULL);
}

__global__ void fill_words(uint64_t* w, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    w[i] = smx(i * 7 + 3) | smx(i * 11 + 5);  // ~75% dense
}

template <int MODE>  // 0 stream, 1 hash, 2 gather, 3 lds
__global__ __launch_bounds__(256) void probe_variant(const int64_t* __restrict__ keys, uint64_t n,
                                                     const uint64_t* __restrict__ words, uint64_t bmask,
                                                     uint64_t* __restrict__ out) {
  __shared__ uint64_t s_masks[1024];
  extern __shared__ uint64_t s_filter[];
  fill_mask_table(s_masks);
  if (MODE == 3)
    for (uint64_t i = threadIdx.x; i <= bmask; i += blockDim.x) s_filter[i] = words[i];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t n_segs = n / 512;
  const uint64_t tw = (uint64_t)gridDim.x * 4;
  uint64_t acc = 0;
  for (uint64_t seg = blockIdx.x * 4ull + (threadIdx.x >> 6); seg < n_segs; seg += tw) {
    uint64_t h[8];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const u64x2 x = *reinterpret_cast<const u64x2*>(keys + seg * 512 + c * 128 + lane * 2);
      h[2 * c] = x[0];
      h[2 * c + 1] = x[1];
    }
    if (MODE == 0) {
#pragma unroll
      for (int j = 0; j < 8; j++) acc ^= h[j];
      continue;
    }
#pragma unroll
    for (int j = 0; j < 8; j++) h[j] = murmur64(h[j]);
    uint64_t pass = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint64_t m = mask_of(s_masks, h[j]);
      uint64_t w;
      if (MODE == 1) w = h[j] | m;
      else if (MODE == 2) w = words[block_of(h[j], bmask)];
      else w = s_filter[block_of(h[j], bmask)];
      pass += ((w & m) == m);
    }
    acc += __popcll(ballot64(pass & 1)) + pass;
  }
  if (acc == 0x123456789ULL) out[0] = acc;  // keep live
}

__global__ void write_buf(uint64_t* b, uint64_t n, uint64_t v) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n / 2; i += (uint64_t)gridDim.x * blockDim.x)
    reinterpret_cast<u64x2*>(b)[i] = u64x2{i ^ v, i + v};
}
__global__ void read_buf(const uint64_t* b, uint64_t n, uint64_t* out) {
  uint64_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n / 2; i += (uint64_t)gridDim.x * blockDim.x) {
    const u64x2 x = reinterpret_cast<const u64x2*>(b)[i];
    acc ^= x[0] + x[1];
  }
  if (acc == 0x1234567ULL) out[0] = acc;
}

template <typename F>
float time_ms(F f, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  f();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; i++) f();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1000000000ULL;
  int cus = 256;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  int64_t* keys;
  uint64_t *words, *out;
  CHECK(hipMalloc(&keys, n * 8));
  CHECK(hipMalloc(&words, (1ULL << 27) * 8));
  CHECK(hipMalloc(&out, 64));
  hipLaunchKernelGGL(gen_keys, dim3(8192), dim3(256), 0, 0, keys, n);
  hipLaunchKernelGGL(fill_words, dim3(8192), dim3(256), 0, 0, words, 1ULL << 27);
  CHECK(hipDeviceSynchronize());
  const unsigned grid = cus * 8;
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(probe_variant<3>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
  auto run = [&](const char* name, int mode, int L, size_t lds, unsigned g) {
    const uint64_t bm = (1ULL << L) - 1;
    float ms = time_ms([&] {
      switch (mode) {
        case 0: hipLaunchKernelGGL(probe_variant<0>, dim3(g), dim3(256), lds, 0, keys, n, words, bm, out); break;
        case 1: hipLaunchKernelGGL(probe_variant<1>, dim3(g), dim3(256), lds, 0, keys, n, words, bm, out); break;
        case 2: hipLaunchKernelGGL(probe_variant<2>, dim3(g), dim3(256), lds, 0, keys, n, words, bm, out); break;
        default: hipLaunchKernelGGL(probe_variant<3>, dim3(g), dim3(256), lds, 0, keys, n, words, bm, out); break;
      }
    }, 5);
    printf("%-8s L=%-2d grid=%-5u %8.3f ms  %7.1f Gkeys/s  key-stream %6.0f GB/s\n", name, L, g, ms, n / ms / 1e6,
           n * 8.0 / ms / 1e6);
  };
  run("stream", 0, 0, 0, grid);
  run("hash", 1, 0, 0, grid);
  for (int L : {10, 13, 15, 17, 18, 19, 20, 21, 22, 24, 27}) run("gather", 2, L, 0, grid);
  for (int L : {10, 12, 13, 14}) run("lds", 3, L, (8ULL << L), cus * (L <= 12 ? 8 : (L == 13 ? 2 : 1)));
  // intermediate buffer residency: write S then read S, repeated
  for (uint64_t S : {16ULL << 20, 64ULL << 20, 128ULL << 20, 192ULL << 20, 512ULL << 20, 4ULL << 30}) {
    const uint64_t nw = S / 8;
    float wms = time_ms([&] { hipLaunchKernelGGL(write_buf, dim3(grid), dim3(256), 0, 0, (uint64_t*)keys, nw, 7); }, 10);
    float rms = time_ms([&] { hipLaunchKernelGGL(read_buf, dim3(grid), dim3(256), 0, 0, (uint64_t*)keys, nw, out); }, 10);
    float wrms = time_ms([&] {
      hipLaunchKernelGGL(write_buf, dim3(grid), dim3(256), 0, 0, (uint64_t*)keys, nw, 7);
      hipLaunchKernelGGL(read_buf, dim3(grid), dim3(256), 0, 0, (uint64_t*)keys, nw, out);
    }, 10);
    printf("mallrw  S=%5llu MiB  write %7.1f GB/s  read %7.1f GB/s  write+read %7.1f GB/s\n",
           (unsigned long long)(S >> 20), S / wms / 1e6, S / rms / 1e6, 2.0 * S / wrms / 1e6);
  }
  CHECK(hipFree(keys));
  CHECK(hipFree(words));
  return 0;
}
