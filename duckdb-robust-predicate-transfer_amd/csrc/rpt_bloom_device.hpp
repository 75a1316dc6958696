// rpt_bloom_device.hpp — device-side arithmetic of the blocked Bloom filter (gfx950).
//
// Spec (Arrow Acero BlockedBloomFilter, the filter the reference README ports, README.md:23-32):
//   mask(h)     = ROTL64(masks.mask(h & 1023), (h >> 10) & 63)   arrow/acero/bloom_filter.h:172-185
//   block_id(h) = (h >> 16) & (num_blocks - 1)                     arrow/acero/bloom_filter.h:187-193
// Key hash (DuckDB VectorOperations::Hash, used by HashColumns, reference src/bloom_filter.cpp:11-24):
//   MurmurHash64 finalizer; int32 keys zero-extended through uint32; NULL rows -> NULL_HASH.
#pragma once

#ifndef RPT_DPP_SCAN
#define RPT_DPP_SCAN 1  // wave prefix sums through DPP (0: ds_bpermute shuffles)
#endif

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rpt {

constexpr int kLogNumMasks = 10;
constexpr int kNumMasks = 1 << kLogNumMasks;
constexpr uint64_t kFullMask = (1ULL << 57) - 1;
constexpr uint64_t kNullHash = 0xbf58476d1ce4e5b9ULL;

// The 136-byte BloomFilterMasks bit vector (arrow/acero/bloom_filter.h:86-90: mask N is the 57 bits
// starting at bit N) as 17 little-endian words, plus one zero word so word w+1 is always readable.
// Checked against the Arrow library's table by tests/test_oracle_golden.py (masks.bin).
__constant__ static const uint64_t kMaskBits[18] = {
    0x4000080001140020ULL, 0x0802000000422000ULL, 0x0040200000808400ULL, 0x0001080000210100ULL,
    0x00000a0000012200ULL, 0x1000000808000240ULL, 0x0804000010002004ULL, 0x0a10000000802001ULL,
    0x0214000000040080ULL, 0x000c200000080200ULL, 0x0200184000000010ULL, 0x4204003000000001ULL,
    0x0044080040000000ULL, 0x1000881000080000ULL, 0x0010011000020000ULL, 0x0000001200100400ULL,
    0x0000000120008808ULL, 0x0000000000000000ULL};

__device__ __forceinline__ uint64_t murmur64(uint64_t x) {
  x ^= x >> 32;
  x *= 0xd6e8feb86659fd93ULL;
  x ^= x >> 32;
  x *= 0xd6e8feb86659fd93ULL;
  x ^= x >> 32;
  return x;
}

// DuckDB CombineHash for composite keys (HashColumns, reference src/bloom_filter.cpp:15-17):
// hashes = CombineHashScalar(hashes, Hash(col_j)) with DuckDB v1.1+'s form: a ^= a >> 32;
// a *= 0xd6e8feb86659fd93; a ^ b (v0.x-1.0: (a * 0xbf58476d1ce4e5b9) ^ b). Restated from DuckDB
// (vector_hash.cpp), not in this container: parity unpinned, as for the key hash itself.
__device__ __forceinline__ uint64_t combine_hash(uint64_t a, uint64_t b) {
  a ^= a >> 32;
  a *= 0xd6e8feb86659fd93ULL;
  return a ^ b;
}

__device__ __forceinline__ uint64_t rotl64(uint64_t x, uint32_t r) {
  return (x << r) | (x >> ((64u - r) & 63u));
}

// Expand the 1024 masks into an 8 KiB LDS table (one ds_read_b64 per key afterwards) -- the direct
// probe and the atomic insert; the slice kernels use the 2048-entry rotated table (partitioned.hpp).
// Must be followed by __syncthreads() before use.
__device__ __forceinline__ void fill_mask_table(uint64_t* s_masks) {
  for (int id = threadIdx.x; id < kNumMasks; id += blockDim.x) {
    const int w = id >> 6, s = id & 63;
    const uint64_t lo = kMaskBits[w], hi = kMaskBits[w + 1];
    s_masks[id] = ((lo >> s) | ((hi << 1) << (63 - s))) & kFullMask;
  }
}

__device__ __forceinline__ uint64_t mask_of(const uint64_t* s_masks, uint64_t h) {
  return rotl64(s_masks[h & (kNumMasks - 1)], static_cast<uint32_t>(h >> kLogNumMasks) & 63u);
}

__device__ __forceinline__ uint64_t block_of(uint64_t h, uint64_t block_mask) {
  return (h >> (kLogNumMasks + 6)) & block_mask;
}

// Key types (rpt_key_type), plus kKeySplit: the bucketed strategy's level-2 input, the low 32 bits
// of each row's hash (keys) with hash bits 32..39 in a parallel byte array (KeyArgs::hi8) -- the 38
// bits a 32 MiB bucket's slices need, in 5 bytes instead of 8.
enum KeyKind : int { kKeyI64 = 0, kKeyI32 = 1, kKeyHash = 2, kKeySplit = 3 };

template <int K> struct KeyTraits;
template <> struct KeyTraits<kKeyI64> {
  using T = int64_t;
  static constexpr int kVec = 2;         // keys per 16-byte load
  static constexpr bool kValues = true;  // key values: validity (NULL_HASH) and min/max apply
  __device__ static __forceinline__ uint64_t hash(T v) { return murmur64(static_cast<uint64_t>(v)); }
};
template <> struct KeyTraits<kKeyI32> {
  using T = int32_t;
  static constexpr int kVec = 4;
  static constexpr bool kValues = true;
  __device__ static __forceinline__ uint64_t hash(T v) {
    return murmur64(static_cast<uint64_t>(static_cast<uint32_t>(v)));
  }
};
template <> struct KeyTraits<kKeyHash> {
  using T = uint64_t;
  static constexpr int kVec = 2;
  static constexpr bool kValues = false;
  __device__ static __forceinline__ uint64_t hash(T v) { return v; }
};
template <> struct KeyTraits<kKeySplit> {
  using T = uint32_t;
  static constexpr int kVec = 4;
  static constexpr bool kValues = false;
  __device__ static __forceinline__ uint64_t hash(T v) { return v; }  // | hi8 << 32, added by the loader
};

// Spread the low 32 bits of x so that bit i lands on bit 2i (wave-uniform: scalar ALU).
__device__ __forceinline__ uint64_t spread2(uint64_t x) {
  x &= 0xffffffffULL;
  x = (x | (x << 16)) & 0x0000FFFF0000FFFFULL;
  x = (x | (x << 8)) & 0x00FF00FF00FF00FFULL;
  x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0FULL;
  x = (x | (x << 2)) & 0x3333333333333333ULL;
  x = (x | (x << 1)) & 0x5555555555555555ULL;
  return x;
}
// Spread the low 16 bits of x so that bit i lands on bit 4i.
__device__ __forceinline__ uint64_t spread4(uint64_t x) {
  x &= 0xffffULL;
  x = (x | (x << 24)) & 0x000000FF000000FFULL;
  x = (x | (x << 12)) & 0x000F000F000F000FULL;
  x = (x | (x << 6)) & 0x0303030303030303ULL;
  x = (x | (x << 3)) & 0x1111111111111111ULL;
  return x;
}

__device__ __forceinline__ uint64_t ballot64(bool p) { return __builtin_amdgcn_ballot_w64(p); }

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
// Set bits of the wave-uniform mask w below this lane.
__device__ __forceinline__ uint32_t mask_rank(uint64_t w) {
  return __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(w >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(w), 0u));
}
// Lane `src`'s 64-bit value, wave-uniform.
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int src) {
  const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(v)), src));
  const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(v >> 32)), src));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}
// Selection-vector expansion of 64 rows whose pass bits are the wave-uniform word w (bit i = row
// row0 + i): lane i writes row i's id at out[rank] if it passes, so one store instruction writes the
// survivors as ONE contiguous run (full lines at high pass rates). Returns the survivor count.
__device__ __forceinline__ uint32_t expand_word_sel(uint64_t w, uint32_t row0, uint32_t lane, const uint32_t* row_sel,
                                                    uint32_t* out) {
  if ((w >> lane) & 1ULL) {
    const uint32_t row = row0 + lane;
    out[mask_rank(w)] = row_sel ? row_sel[row] : row;
  }
  return static_cast<uint32_t>(__popcll(w));
}

// Inclusive wave-wide prefix sum of a 32-bit value (whole wave active). DPP: shifts within rows of 16,
// then row broadcasts 15 / 31 -- six dependent VALU ops instead of six ds_bpermute round trips.
__device__ __forceinline__ uint32_t wave_inclusive_sum(uint32_t v) {
#if RPT_DPP_SCAN
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x111, 0xf, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x112, 0xf, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x114, 0xf, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x118, 0xf, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x142, 0xa, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x143, 0xc, 0xf, false));
  return v;
#else
  const uint32_t lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t o = __shfl_up(v, d, 64);
    if (lane >= static_cast<uint32_t>(d)) v += o;
  }
  return v;
#endif
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

}  // namespace rpt
