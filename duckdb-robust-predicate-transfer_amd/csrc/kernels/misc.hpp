// misc.hpp — atomic insert, hashing, OR merge, popcount, synthetic workload generators.
// Part of librpt_gpu.so: included by rpt_gpu.hip (one translation unit: kernels and their launches
// stay together without relocatable device code).
#pragma once

namespace rpt {

// ---- k2: insert ----------------------------------------------------------------------------------
// v from the lane whose byte address (lane * 4) is src_byte (ds_bpermute on both 32-bit halves)
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src_byte) {
  const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src_byte, static_cast<int>(static_cast<uint32_t>(v))));
  const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src_byte, static_cast<int>(static_cast<uint32_t>(v >> 32))));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

template <int K, bool DENSE>
__global__ __launch_bounds__(kBlockThreads) void insert_kernel(uint64_t* __restrict__ words, uint64_t block_mask,
                                                              KeyArgs a, uint64_t n, uint64_t n_segs,
                                                              int64_t* __restrict__ stats) {
  constexpr bool MM = KeyTraits<K>::kValues;
  __shared__ uint64_t s_masks[kNumMasks];
  fill_mask_table(s_masks);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t total_waves = static_cast<uint64_t>(gridDim.x) * kWavesPerBlock;
  int64_t mm[2] = {kMinInit, kMaxInit};
  for (uint64_t seg = static_cast<uint64_t>(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6); seg < n_segs;
       seg += total_waves) {
    uint64_t h[8];
    bool ok[8];
    load_hashes<K, DENSE, MM>(a, seg * kSegRows, n, lane, h, ok, mm);
    // A row whose hash equals the previous row's sets nothing new: its atomic is dropped. Memory-side atomics
    // on one word serialize at ~11 ns each (a CONSTANT chunk's 2048 equal keys: 37 instead of 13 us per call;
    // 1 Mi equal keys 11.9 ms; profiles/r05/insert_duplicates.jsonl); the previous row is this lane's last
    // hash or the previous lane's (ds_bpermute), lane 0 has none.
    const int src = static_cast<int>(((lane + 63) & 63) << 2);
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint64_t prev;
      bool has_prev;
      if constexpr (DENSE && KeyTraits<K>::kVec > 1) {
        constexpr int V = KeyTraits<K>::kVec;
        if (j % V != 0) {
          prev = h[j - 1];
          has_prev = true;
        } else {
          prev = shfl_u64(h[j + V - 1], src);
          has_prev = lane != 0;
        }
      } else {
        prev = shfl_u64(h[j], src);
        has_prev = lane != 0;
      }
      if (ok[j] && !(has_prev && prev == h[j])) {
        __hip_atomic_fetch_or(words + block_of(h[j], block_mask), mask_of(s_masks, h[j]), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if constexpr (MM) {
    wave_minmax(mm[0], mm[1]);
    publish_minmax(mm[0], mm[1], stats);
  }
}

// ---- hashing only (parity / debugging) ---------------------------------------------------------
template <int K, bool COMBINE>
__global__ __launch_bounds__(kBlockThreads) void hash_kernel(KeyArgs a, uint64_t n, uint64_t* __restrict__ out) {
  using Tr = KeyTraits<K>;
  const typename Tr::T* keys = static_cast<const typename Tr::T*>(a.keys);
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint64_t k = a.key_sel ? a.key_sel[i] : i;
    uint64_t hv = Tr::hash(keys[k]);
    if (KeyTraits<K>::kValues && !valid_at(a.validity, k)) hv = kNullHash;
    out[i] = COMBINE ? combine_hash(out[i], hv) : hv;
  }
}

// ---- k4: OR merge --------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlockThreads) void or_slices_kernel(uint64_t* __restrict__ dst,
                                                                 const uint64_t* __restrict__ srcs, uint32_t k,
                                                                 uint64_t n_words, uint64_t src_stride,
                                                                 int accumulate) {
  // srcs: k slices of n_words words, slice s at srcs + s * src_stride (dst and every slice 16-B aligned)
  const uint64_t n_pairs = n_words / 2;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n_pairs; i += stride) {
    u64x2 acc = accumulate ? reinterpret_cast<const u64x2*>(dst)[i] : u64x2{0, 0};
    for (uint32_t s = 0; s < k; s++) acc |= reinterpret_cast<const u64x2*>(srcs + s * src_stride)[i];
    reinterpret_cast<u64x2*>(dst)[i] = acc;
  }
  if ((n_words & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    uint64_t acc = accumulate ? dst[n_words - 1] : 0ULL;
    for (uint32_t s = 0; s < k; s++) acc |= srcs[s * src_stride + n_words - 1];
    dst[n_words - 1] = acc;
  }
}

// ---- narrow BIGINT keys: 4-B low words + one high word per chunk -> int64 keys --------------------
// One workgroup per chunk c (rows [row0[c], row0[c + 1])): out[r] = hi[c] << 32 | lo[r]. The host-to-device copy of
// a host-resident batch is the bound of the DuckDB shim; BIGINT keys whose chunk shares its high 32 bits
// cross PCIe as 4 B and are widened here (HBM: 12 B per key, microseconds per stage).
constexpr int kWidenThreads = 256;
__global__ __launch_bounds__(kWidenThreads) void widen_keys_kernel(const uint32_t* __restrict__ lo,
                                                                  const uint32_t* __restrict__ hi,
                                                                  const uint32_t* __restrict__ row0,
                                                                  uint64_t* __restrict__ out) {
  const uint32_t c = blockIdx.x;
  const uint32_t a = row0[c], e = row0[c + 1];
  const uint64_t h = static_cast<uint64_t>(hi[c]) << 32;
  for (uint32_t r = a + threadIdx.x; r < e; r += kWidenThreads) out[r] = h | lo[r];
}

// ---- popcount ------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlockThreads) void popcount_kernel(const uint64_t* __restrict__ w, uint64_t n_words,
                                                                unsigned long long* __restrict__ out) {
  __shared__ uint32_t s_part[kWavesPerBlock];
  uint32_t s = 0;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n_words;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    s += __popcll(w[i]);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(out, static_cast<unsigned long long>(s_part[0]) + s_part[1] + s_part[2] + s_part[3]);
  }
}

// ---- word equality (BlockedBloomFilter::IsSameAs) -------------------------------------------------
// Number of word positions where a and b differ, 16-B loads (both 16-B aligned: filters are hipMalloc'd).
__global__ __launch_bounds__(kBlockThreads) void diff_count_kernel(const uint64_t* __restrict__ a,
                                                                  const uint64_t* __restrict__ b, uint64_t n_words,
                                                                  unsigned long long* __restrict__ out) {
  __shared__ uint32_t s_part[kWavesPerBlock];
  uint32_t d = 0;
  const uint64_t n_pairs = n_words / 2;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n_pairs; i += stride) {
    const u64x2 x = reinterpret_cast<const u64x2*>(a)[i], y = reinterpret_cast<const u64x2*>(b)[i];
    d += (x[0] != y[0]) + (x[1] != y[1]);
  }
  if ((n_words & 1) && blockIdx.x == 0 && threadIdx.x == 0) d += a[n_words - 1] != b[n_words - 1];
  d = wave_sum(d);
  if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = d;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = s_part[0] + s_part[1] + s_part[2] + s_part[3];
    if (t) atomicAdd(out, static_cast<unsigned long long>(t));
  }
}

// ---- stream calibration (bench.py: the box's achievable HBM rates beside the kernels' fractions) --
// The fastest of the variants tools/ubench/ubench_stream.hip measured (profiles/r06/ubench_stream.txt):
// read: grid-stride 16-B non-temporal loads, 8 in flight per lane, 16 x 256-thread workgroups per CU (6.6 TB/s),
// folded into one word per workgroup (written, so nothing is dead code); copy: a one-shot grid, one 16-B unit per
// lane, non-temporal store (6.3 TB/s of read + write bytes; a grid-stride copy reached only 4.9).
constexpr int kStreamUnroll = 8;
constexpr int kStreamBlocksPerCU = 16;
__global__ __launch_bounds__(kBlockThreads) void stream_read_kernel(const u64x2* __restrict__ src, uint64_t n16,
                                                                   uint64_t* __restrict__ sink) {
  __shared__ uint64_t s_part[kWavesPerBlock];
  u64x2 acc = {0, 0};
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i + (kStreamUnroll - 1) * stride < n16; i += kStreamUnroll * stride) {
    u64x2 v[kStreamUnroll];
#pragma unroll
    for (int u = 0; u < kStreamUnroll; u++) v[u] = __builtin_nontemporal_load(src + i + u * stride);
#pragma unroll
    for (int u = 0; u < kStreamUnroll; u++) acc ^= v[u];
  }
  for (; i < n16; i += stride) acc ^= __builtin_nontemporal_load(src + i);
  uint64_t x = acc[0] ^ acc[1];
  for (int off = 32; off > 0; off >>= 1) x ^= shfl_u64(x, static_cast<int>(((threadIdx.x + off) & 63) << 2));
  if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x == 0) sink[blockIdx.x] = s_part[0] ^ s_part[1] ^ s_part[2] ^ s_part[3];
}

__global__ __launch_bounds__(kBlockThreads) void stream_copy_kernel(const u64x2* __restrict__ src, uint64_t n16,
                                                                   u64x2* __restrict__ dst) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n16) __builtin_nontemporal_store(src[i], dst + i);
}

// ---- synthetic workload (bench / tests) ----------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t sm64(uint64_t seed, uint64_t i) { return mix64(seed + (i + 1) * 0x9e3779b97f4a7c15ULL); }

__global__ __launch_bounds__(kBlockThreads) void synth_build_kernel(int64_t* __restrict__ out, uint64_t start,
                                                                   uint64_t n) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    out[i] = static_cast<int64_t>(sm64(RPT_SYNTH_SEED_BUILD, start + i));
}

__global__ __launch_bounds__(kBlockThreads) void synth_probe_kernel(int64_t* __restrict__ out, uint64_t n_build,
                                                                   uint32_t p_permille, uint64_t start, uint64_t n) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint64_t r = start + i;
    const uint64_t u = sm64(RPT_SYNTH_SEED_PROBE_SEL, r);
    out[i] = (n_build > 0 && (u % 1000) < p_permille)
                 ? static_cast<int64_t>(sm64(RPT_SYNTH_SEED_BUILD, (u >> 20) % n_build))
                 : static_cast<int64_t>(sm64(RPT_SYNTH_SEED_PROBE_MISS, r));
  }
}
}  // namespace rpt
