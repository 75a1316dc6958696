// ubench_skeleton — the direct probe's memory skeleton without its arithmetic: why does the int64 LDS probe with
// neither hash nor filter lookups (RPT_EXP_PROBE_NO_HASH: 1.575 ms per 1e9 keys, profiles/r06/ab_probe_bound.txt)
// stream its 8 GB at ~5.1 TB/s when a plain read stream reaches ~6.5?
// Each variant reads 1e9 int64 keys with 16-B non-temporal loads in 512-row segments (4 KiB per wave, the probe's
// RawSeg layout), takes pass = a key bit, ballots the 8 pass flags and stores the segment's 8 result words (lanes
// 0-7) + its count (lane 0), as store_segment_bits does.
//   T        : threads per workgroup (1024 = the LDS probe's, 256 = the gather probe's)
//   G        : workgroups per CU
//   NB       : segments in flight per wave (2 = the product's ping-pong: the next segment loads while this one is
//              used; 3, 4: deeper)
//   order    : "strided" = the product's (wave w of workgroup b takes segments b * W + w, + all waves);
//              "blocked" = each wave takes a contiguous run of segments
//   stores   : 1 = result words + counts stored, 0 = folded into a sink
// Best of 7, HIP events. Tools only; not the product.
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
constexpr uint64_t kSegRows = 512;

struct Seg {
  u64x2 r[4];
  __device__ __forceinline__ void load(const u64x2* keys, uint64_t seg, uint32_t lane) {
    const u64x2* kb = keys + seg * (kSegRows / 2) + lane;
#pragma unroll
    for (int c = 0; c < 4; c++) r[c] = __builtin_nontemporal_load(kb + c * 64);
  }
};

template <int T, int NB, bool STORES, bool BLOCKED>
__global__ __launch_bounds__(T) void skeleton(const u64x2* __restrict__ keys, uint64_t n_segs, uint64_t* __restrict__ bits,
                                              uint32_t* __restrict__ counts, uint64_t* __restrict__ sink) {
  constexpr uint32_t W = T / 64;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = static_cast<uint64_t>(blockIdx.x) * W + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t total_waves = static_cast<uint64_t>(gridDim.x) * W;
  uint64_t first, step, end;
  if (BLOCKED) {
    const uint64_t per = (n_segs + total_waves - 1) / total_waves;
    first = wave * per;
    end = first + per < n_segs ? first + per : n_segs;
    step = 1;
  } else {
    first = wave;
    end = n_segs;
    step = total_waves;
  }
  Seg R[NB];
  uint64_t acc = 0;
#pragma unroll
  for (int b = 0; b < NB - 1; b++) {
    const uint64_t s = first + b * step;
    R[b].load(keys, s < end ? s : first, lane);
  }
  uint64_t seg = first;
  bool more = seg < end;
  while (more) {
#pragma unroll
    for (int b = 0; b < NB; b++) {
      if (more) {
        const uint64_t nx = seg + (NB - 1) * step;
        R[(b + NB - 1) % NB].load(keys, nx < end ? nx : first, lane);
        asm volatile("" ::: "memory");
        uint64_t word[8];
        uint32_t cnt = 0;
#pragma unroll
        for (int c = 0; c < 4; c++)
#pragma unroll
          for (int e = 0; e < 2; e++) {
            word[c * 2 + e] = __builtin_amdgcn_ballot_w64((R[b].r[c][e] >> 7) & 1);
            cnt += __popcll(word[c * 2 + e]);
          }
        uint64_t mine = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) mine = lane == static_cast<uint32_t>(j) ? word[j] : mine;
        if (STORES) {
          if (lane < 8) bits[seg * 8 + lane] = mine;
          if (lane == 0) counts[seg] = cnt;
        } else {
          acc += mine + cnt;
        }
        seg += step;
        more = seg < end;
      }
    }
  }
  if (!STORES && acc == 0x123456789ULL) sink[0] = acc;
}


// blocked order, result words of 8 consecutive segments gathered in one register per lane (lane 8j + w = word w of
// the batch's segment j) and written as one 512-B store; counts of 64 segments as one 256-B store
template <int T, int NB>
__global__ __launch_bounds__(T) void skeleton_batched(const u64x2* __restrict__ keys, uint64_t n_segs,
                                                      uint64_t* __restrict__ bits, uint32_t* __restrict__ counts,
                                                      uint64_t* __restrict__ sink) {
  constexpr uint32_t W = T / 64;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = static_cast<uint64_t>(blockIdx.x) * W + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t total_waves = static_cast<uint64_t>(gridDim.x) * W;
  // runs of whole 64-segment blocks per wave (the tail: whatever is left, handled the same way with bounds)
  const uint64_t blocks = (n_segs + 63) / 64;
  const uint64_t per = (blocks + total_waves - 1) / total_waves;
  const uint64_t first = wave * per * 64;
  const uint64_t end = first + per * 64 < n_segs ? first + per * 64 : n_segs;
  if (first >= end) return;
  Seg R[NB];
#pragma unroll
  for (int b = 0; b < NB - 1; b++) {
    const uint64_t s = first + b;
    R[b].load(keys, s < end ? s : first, lane);
  }
  uint64_t seg = first;
  uint64_t wbuf = 0;
  uint32_t cbuf = 0;
  bool more = true;
  while (more) {
#pragma unroll
    for (int b = 0; b < NB; b++) {
      if (more) {
        const uint64_t nx = seg + (NB - 1);
        R[(b + NB - 1) % NB].load(keys, nx < end ? nx : first, lane);
        asm volatile("" ::: "memory");
        uint64_t word[8];
        uint32_t cnt = 0;
#pragma unroll
        for (int c = 0; c < 4; c++)
#pragma unroll
          for (int e = 0; e < 2; e++) {
            word[c * 2 + e] = __builtin_amdgcn_ballot_w64((R[b].r[c][e] >> 7) & 1);
            cnt += __popcll(word[c * 2 + e]);
          }
        const uint32_t j = static_cast<uint32_t>(seg & 7);
#pragma unroll
        for (int w = 0; w < 8; w++) wbuf = lane == j * 8 + w ? word[w] : wbuf;
        cbuf = lane == static_cast<uint32_t>(seg & 63) ? cnt : cbuf;
        if (j == 7 || seg + 1 == end) {
          const uint64_t s0 = seg & ~7ULL;
          if (s0 * 8 + lane < (seg + 1) * 8) bits[s0 * 8 + lane] = wbuf;
        }
        if ((seg & 63) == 63 || seg + 1 == end) {
          const uint64_t c0 = seg & ~63ULL;
          if (c0 + lane <= seg) counts[c0 + lane] = cbuf;
        }
        seg += 1;
        more = seg < end;
      }
    }
  }
}

// the product's structure (strided, NB = 2), the stores made unconditional: buffer stores whose descriptor covers only
// the segment's 8 words (count: 4 bytes), so lanes past them are dropped by the range check instead of being skipped
// by a branch (a skipped store leaves the compiler's memory counter unknown: it waits for everything, s_waitcnt
// vmcnt(0), before each segment's data)
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
constexpr int kRsrcWord3 = 0x00020000;  // gfx9 raw buffer: 32-bit data format, no swizzle
template <int T, int NB>
__global__ __launch_bounds__(T) void skeleton_bufstore(const u64x2* __restrict__ keys, uint64_t n_segs,
                                                       uint64_t* __restrict__ bits, uint32_t* __restrict__ counts,
                                                       uint64_t* __restrict__ sink) {
  constexpr uint32_t W = T / 64;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t first = static_cast<uint64_t>(blockIdx.x) * W + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * W, end = n_segs;
  Seg R[NB];
#pragma unroll
  for (int b = 0; b < NB - 1; b++) {
    const uint64_t s = first + b * step;
    R[b].load(keys, s < end ? s : first, lane);
  }
  uint64_t seg = first;
  bool more = seg < end;
  while (more) {
#pragma unroll
    for (int b = 0; b < NB; b++) {
      if (more) {
        const uint64_t nx = seg + (NB - 1) * step;
        R[(b + NB - 1) % NB].load(keys, nx < end ? nx : first, lane);
        asm volatile("" ::: "memory");
        uint64_t word[8];
        uint32_t cnt = 0;
#pragma unroll
        for (int c = 0; c < 4; c++)
#pragma unroll
          for (int e = 0; e < 2; e++) {
            word[c * 2 + e] = __builtin_amdgcn_ballot_w64((R[b].r[c][e] >> 7) & 1);
            cnt += __popcll(word[c * 2 + e]);
          }
        uint64_t mine = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) mine = lane == static_cast<uint32_t>(j) ? word[j] : mine;
        const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(bits + seg * 8, 0, 64, kRsrcWord3);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{static_cast<uint32_t>(mine), static_cast<uint32_t>(mine >> 32)}, rw,
                                              static_cast<int>(lane * 8), 0, 0);
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(counts + seg, 0, 4, kRsrcWord3);
        __builtin_amdgcn_raw_buffer_store_b32(cnt, rc, static_cast<int>(lane * 4), 0, 0);
        seg += step;
        more = seg < end;
      }
    }
  }
}

// the product's structure with the stores varied: MODE 1 = non-temporal stores, MODE 2 = plain stores into a 4 MiB
// ring of result words (counts: 256 KiB) that stays in the caches -- does the cost come from writing to HBM?
template <int T, int MODE, int RING_LOG = 16>
__global__ __launch_bounds__(T) void skeleton_storemode(const u64x2* __restrict__ keys, uint64_t n_segs,
                                                        uint64_t* __restrict__ bits, uint32_t* __restrict__ counts,
                                                        uint64_t* __restrict__ sink) {
  constexpr uint32_t W = T / 64;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t first = static_cast<uint64_t>(blockIdx.x) * W + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * W, end = n_segs;
  Seg R[2];
  R[0].load(keys, first < end ? first : 0, lane);
  uint64_t seg = first;
  bool more = seg < end;
  while (more) {
#pragma unroll
    for (int b = 0; b < 2; b++) {
      if (more) {
        const uint64_t nx = seg + step;
        R[(b + 1) % 2].load(keys, nx < end ? nx : first, lane);
        asm volatile("" ::: "memory");
        uint64_t word[8];
        uint32_t cnt = 0;
#pragma unroll
        for (int c = 0; c < 4; c++)
#pragma unroll
          for (int e = 0; e < 2; e++) {
            word[c * 2 + e] = __builtin_amdgcn_ballot_w64((R[b].r[c][e] >> 7) & 1);
            cnt += __popcll(word[c * 2 + e]);
          }
        uint64_t mine = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) mine = lane == static_cast<uint32_t>(j) ? word[j] : mine;
        const uint64_t ws = MODE == 2 ? (seg & ((1ULL << RING_LOG) - 1)) : seg;
        if (lane < 8) {
          if (MODE == 1) __builtin_nontemporal_store(mine, bits + ws * 8 + lane);
          else bits[ws * 8 + lane] = mine;
        }
        if (lane == 0) {
          if (MODE == 1) __builtin_nontemporal_store(cnt, counts + ws);
          else counts[ws] = cnt;
        }
        seg += step;
        more = seg < end;
      }
    }
  }
}

__global__ void fill(uint64_t* k, uint64_t n) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) k[i] = i * 0x9e3779b97f4a7c15ULL;
}
__global__ __launch_bounds__(256) void k_read(const u64x2* __restrict__ src, uint64_t n16, uint64_t* sink) {
  u64x2 acc = {0, 0};
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i + 7 * stride < n16; i += 8 * stride) {
    u64x2 v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) v[u] = __builtin_nontemporal_load(src + i + u * stride);
#pragma unroll
    for (int u = 0; u < 8; u++) acc ^= v[u];
  }
  for (; i < n16; i += stride) acc ^= src[i];
  if ((acc[0] ^ acc[1]) == 0x123456789ULL) sink[0] = 1;
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
    best = std::min(best, static_cast<double>(ms));
  }
  return best;
}

int main() {
  const uint64_t n = 1000000000ULL, n_segs = n / kSegRows;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint64_t *keys, *bits, *sink;
  uint32_t* counts;
  CK(hipMalloc(&keys, n * 8));
  CK(hipMalloc(&bits, n_segs * 64));
  CK(hipMalloc(&counts, n_segs * 4));
  CK(hipMalloc(&sink, 8));
  hipLaunchKernelGGL(fill, dim3((n + 255) / 256), dim3(256), 0, 0, keys, n);
  const u64x2* k2 = reinterpret_cast<const u64x2*>(keys);
  const double gb = n * 8 / 1e9;
  double ms = best_ms([&] { hipLaunchKernelGGL(k_read, dim3(cus * 16), dim3(256), 0, 0, k2, n / 2, sink); });
  printf("%-44s %.3f ms  %5.0f GB/s\n", "read stream (16 x 256 per CU, 8 in flight)", ms, gb / ms * 1e3);
  auto run = [&](const char* name, auto kern, int T, int G) {
    const double t = best_ms([&] { hipLaunchKernelGGL(kern, dim3(cus * G), dim3(T), 0, 0, k2, n_segs, bits, counts, sink); });
    printf("%-36s T=%4d G=%d %.3f ms  %5.0f GB/s\n", name, T, G, t, gb / t * 1e3);
  };
  run("strided NB=2 stores (product)", skeleton<1024, 2, true, false>, 1024, 1);
  run("strided NB=2 no stores", skeleton<1024, 2, false, false>, 1024, 1);
  run("strided NB=3 stores", skeleton<1024, 3, true, false>, 1024, 1);
  run("strided NB=4 stores", skeleton<1024, 4, true, false>, 1024, 1);
  run("blocked NB=2 stores", skeleton<1024, 2, true, true>, 1024, 1);
  run("blocked NB=3 stores", skeleton<1024, 3, true, true>, 1024, 1);
  run("strided NB=2 stores", skeleton<1024, 2, true, false>, 1024, 2);
  run("strided NB=2 stores", skeleton<256, 2, true, false>, 256, 8);
  run("strided NB=3 stores", skeleton<256, 3, true, false>, 256, 8);
  run("strided NB=2 no stores", skeleton<256, 2, false, false>, 256, 8);
  run("blocked NB=2 stores", skeleton<256, 2, true, true>, 256, 8);
  run("strided NB=2 stores", skeleton<256, 2, true, false>, 256, 16);
  run("blocked NB=2 batched stores", skeleton_batched<1024, 2>, 1024, 1);
  run("blocked NB=3 batched stores", skeleton_batched<1024, 3>, 1024, 1);
  run("blocked NB=2 batched stores", skeleton_batched<256, 2>, 256, 8);
  run("blocked NB=3 batched stores", skeleton_batched<256, 3>, 256, 8);
  run("strided NB=2 buffer stores", skeleton_bufstore<1024, 2>, 1024, 1);
  run("strided NB=2 plain stores (mode 0)", skeleton_storemode<1024, 0>, 1024, 1);
  run("strided NB=2 nt stores", skeleton_storemode<1024, 1>, 1024, 1);
  run("strided NB=2 stores into 4 MiB ring", skeleton_storemode<1024, 2>, 1024, 1);
  // rings of 2^L segments' 64-B words: 16 / 32 / 64 / 128 MiB
  run("stores into 16 MiB ring", skeleton_storemode<1024, 2, 18>, 1024, 1);
  run("stores into 32 MiB ring", skeleton_storemode<1024, 2, 19>, 1024, 1);
  run("stores into 64 MiB ring", skeleton_storemode<1024, 2, 20>, 1024, 1);
  run("stores into 128 MiB ring", skeleton_storemode<1024, 2, 21>, 1024, 1);
  run("strided NB=2 nt stores", skeleton_storemode<256, 1>, 256, 8);
  run("strided NB=2 stores into 4 MiB ring", skeleton_storemode<256, 2>, 256, 8);
  run("strided NB=3 buffer stores", skeleton_bufstore<1024, 3>, 1024, 1);
  run("strided NB=2 buffer stores", skeleton_bufstore<256, 2>, 256, 8);
  // check the batched kernel's words and counts against the plain one
  uint64_t* bits2;
  uint32_t* counts2;
  CK(hipMalloc(&bits2, n_segs * 64));
  CK(hipMalloc(&counts2, n_segs * 4));
  hipLaunchKernelGGL((skeleton<1024, 2, true, false>), dim3(cus), dim3(1024), 0, 0, k2, n_segs, bits, counts, sink);
  hipLaunchKernelGGL((skeleton_bufstore<1024, 2>), dim3(cus), dim3(1024), 0, 0, k2, n_segs, bits2, counts2, sink);
  CK(hipDeviceSynchronize());
  uint64_t* hb = static_cast<uint64_t*>(malloc(n_segs * 64));
  uint64_t* hb2 = static_cast<uint64_t*>(malloc(n_segs * 64));
  uint32_t* hc = static_cast<uint32_t*>(malloc(n_segs * 4));
  uint32_t* hc2 = static_cast<uint32_t*>(malloc(n_segs * 4));
  CK(hipMemcpy(hb, bits, n_segs * 64, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hb2, bits2, n_segs * 64, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hc, counts, n_segs * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hc2, counts2, n_segs * 4, hipMemcpyDeviceToHost));
  uint64_t bad = 0;
  for (uint64_t i = 0; i < n_segs * 8; i++) bad += hb[i] != hb2[i];
  for (uint64_t i = 0; i < n_segs; i++) bad += hc[i] != hc2[i];
  printf("buffer-store vs plain: %llu mismatches\n", (unsigned long long)bad);
  return 0;
}
