// rpt_gpu.hip — HIP kernels (gfx950) and the C-ABI of librpt_gpu.so (include/rpt_gpu.h).
//
// Hot path: PTBloomFilter::Insert / LookupSel (reference src/bloom_filter.cpp:60-78),
// called per DataChunk by PhysicalCreateBF::Sink (physical_create_bf.cpp:221-227) and
// PhysicalUseBF::ExecuteInternal (physical_use_bf.cpp:163). Re-designed for MI355X:
//
//   insert   : one pass over the key column, 16-B coalesced loads, hash in registers, mask from an
//              8 KiB LDS table, one device-scope 64-bit atomic OR per key (k2).
//   probe    : P1 hash + gather + wave ballot -> result bit vector (Arrow Find layout) + one
//              survivor count per 512-row wave segment;  P2 two-level scan of the counts;
//              P3 expand bits into an ascending uint32 selection vector (k1).
//   merge    : OR of partial filters / peer slices (k4);  fold (k3);  popcount.
//
// All kernels are persistent grid-stride loops over 512-row wave segments: a wave owns a segment
// end to end, so P1 needs no barrier after the LDS mask-table fill.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "rpt_bloom_device.hpp"
#include "rpt_gpu.h"
#include "rpt_gpu_synth.h"

namespace rpt {

constexpr int kBlockThreads = 256;
constexpr int kWavesPerBlock = kBlockThreads / 64;
constexpr uint64_t kSegRows = 512;                 // rows per wave segment (8 per lane)
constexpr uint64_t kWordsPerSeg = kSegRows / 64;   // result-bit words per segment
constexpr uint64_t kGroupSegs = 256;               // segments per scan group (one compaction workgroup)
constexpr int kBlocksPerCU = 8;

// Partitioned ("routed") probe: the filter is cut into 128 KiB slices that fit in LDS; probe rows are
// bucketed by slice per 16 Ki-row tile so that every filter access is an LDS read.
#ifndef RPT_SLICE_LOG
#define RPT_SLICE_LOG 14
#endif
constexpr int kSliceLog = RPT_SLICE_LOG;               // 2^13 blocks = 64 KiB (or 2^14 = 128 KiB) per slice
constexpr uint64_t kSliceWords = 1ULL << kSliceLog;
constexpr int kMaxSliceCount = 1024;                   // P <= 1024 slices (filters <= 128 MiB at 128 KiB slices)
#ifndef RPT_TILE_ROWS
#define RPT_TILE_ROWS 16384
#endif
constexpr uint64_t kTileRows = RPT_TILE_ROWS;          // rows per partition tile (8 or 16 per thread)
// Runs are padded to kRunPad records so a lane owns kRunPad aligned records of one run and its pass
// results form one byte of bits. Tile capacity is a multiple of 128 so the tile's pass bits are
// whole 16-byte vectors.
constexpr uint32_t kRunPad = 8;
__host__ __device__ constexpr uint32_t pad_run(uint32_t c) { return (c + kRunPad - 1) & ~(kRunPad - 1); }
__host__ __device__ constexpr uint64_t tile_cap_for(uint32_t n_slices) {
  return (kTileRows + static_cast<uint64_t>(kRunPad) * n_slices + 127) & ~127ULL;
}
// Bucketed strategy (filters > 128 MiB): 16 MiB buckets of 128 slices, at most 1024 buckets (16 GiB).
constexpr int kBucketSliceLog = 7;
constexpr uint32_t kBucketSlices = 1u << kBucketSliceLog;
constexpr uint32_t kMaxBuckets = 1024;
constexpr int kTileThreads = 1024;                     // 16 waves
constexpr int kRowsPerThread = static_cast<int>(kTileRows / kTileThreads);
constexpr int kSegsPerWaveA = kRowsPerThread / 8;      // 512-row segments per wave in the partition kernel
static_assert(kRowsPerThread == 8 || kRowsPerThread == 16 || kRowsPerThread == 32, "tile = 8, 16 or 32 Ki rows");
constexpr int kSliceThreads = 1024;                    // slice-probe workgroup (16 waves)
constexpr int kLdsDirectMaxLog = 13;                   // filters <= 64 KiB: whole filter in LDS
#ifndef RPT_SLICE_UNROLL
#define RPT_SLICE_UNROLL 4                             // 512-record steps in flight per wave
#endif
#ifndef RPT_PARTITION_MIN_WAVES
#define RPT_PARTITION_MIN_WAVES 8                      // 2 partition workgroups per CU (64 VGPRs)
#endif

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct KeyArgs {
  const void* keys;
  const uint32_t* key_sel;
  const uint64_t* validity;
  const uint32_t* row_sel;
};

__device__ __forceinline__ bool valid_at(const uint64_t* validity, uint64_t idx) {
  return validity == nullptr || ((validity[idx >> 6] >> (idx & 63)) & 1ULL);
}

// Hashes of the 8 rows a lane owns in a segment.
//  DENSE   (flat column, no selections, 16-B aligned): row(c, e) = base + c*64*V + lane*V + e,
//          one 16-byte load per (c): fully coalesced 1 KiB per wave instruction.
//  GENERAL (dictionary key_sel and/or row_sel):        row(c) = base + c*64 + lane.
// MM: also fold the valid (non-NULL, in-range) key values into mm[0] = min, mm[1] = max (the build's
// min/max dynamic filter, physical_create_bf.cpp:82-119, fused into the key read).
template <int K, bool DENSE, bool MM = false>
__device__ __forceinline__ void load_hashes(const KeyArgs& a, uint64_t base, uint64_t n, uint32_t lane,
                                            uint64_t (&h)[8], bool (&ok)[8], int64_t* mm = nullptr) {
  using Tr = KeyTraits<K>;
  using T = typename Tr::T;
  // rows left from `base` (uniform), so per-row bounds checks are 32-bit and addresses are
  // uniform-base + 32-bit lane offset
  const uint32_t rem = n > base ? static_cast<uint32_t>(n - base < kSegRows ? n - base : kSegRows) : 0u;
  if constexpr (DENSE) {
    constexpr int V = Tr::kVec;
    const T* kb = static_cast<const T*>(a.keys) + base;
    const uint64_t* vb = a.validity ? a.validity + (base >> 6) : nullptr;  // base is a multiple of 512
#pragma unroll
    for (int c = 0; c < 8 / V; c++) {
      const uint32_t off = static_cast<uint32_t>(c * 64 * V) + lane * V;
      T v[V];
      if (off + V <= rem) {
        if constexpr (V == 2) {
          const u64x2 x = *reinterpret_cast<const u64x2*>(kb + off);
          v[0] = static_cast<T>(x[0]);
          v[1] = static_cast<T>(x[1]);
        } else {
          const u32x4 x = *reinterpret_cast<const u32x4*>(kb + off);
#pragma unroll
          for (int e = 0; e < V; e++) v[e] = static_cast<T>(x[e]);
        }
      } else {
#pragma unroll
        for (int e = 0; e < V; e++) v[e] = (off + e < rem) ? kb[off + e] : T(0);
      }
      // validity bits of this lane's V rows, shifted down to bits 0..V-1 (V | 64: one word)
      uint32_t vbits = (1u << V) - 1;
      if (K != kKeyHash && vb != nullptr && off < rem) vbits = static_cast<uint32_t>(vb[off >> 6] >> (off & 63));
#pragma unroll
      for (int e = 0; e < V; e++) {
        ok[c * V + e] = off + e < rem;
        uint64_t hv = Tr::hash(v[e]);
        if (K != kKeyHash && !((vbits >> e) & 1u)) hv = kNullHash;
        h[c * V + e] = hv;
        if constexpr (MM && K != kKeyHash) {
          if (off + e < rem && ((vbits >> e) & 1u)) {
            mm[0] = min(mm[0], static_cast<int64_t>(v[e]));
            mm[1] = max(mm[1], static_cast<int64_t>(v[e]));
          }
        }
      }
    }
  } else {
    const T* keys = static_cast<const T*>(a.keys);
#pragma unroll
    for (int c = 0; c < 8; c++) {
      const uint32_t off = static_cast<uint32_t>(c * 64) + lane;
      ok[c] = off < rem;
      uint64_t hv = 0;
      if (ok[c]) {
        const uint64_t i = base + off;
        const uint64_t r = a.row_sel ? a.row_sel[i] : i;
        const uint64_t k = a.key_sel ? a.key_sel[r] : r;
        const T kv = keys[k];
        hv = Tr::hash(kv);
        const bool valid = valid_at(a.validity, k);
        if (K != kKeyHash && !valid) hv = kNullHash;
        if constexpr (MM && K != kKeyHash) {
          if (valid) {
            mm[0] = min(mm[0], static_cast<int64_t>(kv));
            mm[1] = max(mm[1], static_cast<int64_t>(kv));
          }
        }
      }
      h[c] = hv;
    }
  }
}

// Row offset inside a 512-row segment of the j-th hash load_hashes<K, DENSE> returns for `lane`.
template <int K, bool DENSE>
__device__ __forceinline__ uint32_t seg_row(int j, uint32_t lane) {
  if constexpr (DENSE) {
    constexpr int V = KeyTraits<K>::kVec;
    return static_cast<uint32_t>((j / V) * 64 * V) + lane * V + static_cast<uint32_t>(j % V);
  } else {
    return static_cast<uint32_t>(j * 64) + lane;
  }
}

// Wave-wide (min, max) of per-lane values, returned wave-uniform (scalar registers).
__device__ __forceinline__ void wave_minmax(int64_t& mn, int64_t& mx) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    mn = min(mn, static_cast<int64_t>(__shfl_xor(static_cast<long long>(mn), d, 64)));
    mx = max(mx, static_cast<int64_t>(__shfl_xor(static_cast<long long>(mx), d, 64)));
  }
  auto uniform = [](int64_t v) {
    const uint64_t u = static_cast<uint64_t>(v);
    const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(u));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(u >> 32));
    return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
  };
  mn = uniform(mn);
  mx = uniform(mx);
}
// Fold a wave's uniform (min, max) into stats[0..1] (int64, device). A wave whose values cannot lower
// the min or raise the max — the common case once a few waves have reported — skips the atomics.
__device__ __forceinline__ void publish_minmax(int64_t mn, int64_t mx, int64_t* stats) {
  if ((threadIdx.x & 63) == 0) {
    if (mn < __hip_atomic_load(stats, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      __hip_atomic_fetch_min(stats, mn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (mx > __hip_atomic_load(stats + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      __hip_atomic_fetch_max(stats + 1, mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
constexpr int64_t kMinInit = INT64_MAX, kMaxInit = INT64_MIN;  // "no value yet"

// ---- P1: probe -> result bits + per-segment survivor counts ------------------------------------
// FILTER_IN_LDS: the whole filter (<= 64 KiB) is staged in LDS and every gather is an LDS read.
template <int K, bool DENSE, bool FILTER_IN_LDS>
__global__ __launch_bounds__(kBlockThreads) void probe_bits_kernel(const uint64_t* __restrict__ words,
                                                                  uint64_t block_mask, KeyArgs a, uint64_t n,
                                                                  uint64_t n_segs, uint64_t* __restrict__ out_bits,
                                                                  uint32_t* __restrict__ seg_counts) {
  __shared__ uint64_t s_masks[kNumMasks];
  extern __shared__ uint64_t s_filter[];
  fill_mask_table(s_masks);
  if constexpr (FILTER_IN_LDS) {
    for (uint64_t i = threadIdx.x; i <= block_mask; i += blockDim.x) s_filter[i] = words[i];
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t total_waves = static_cast<uint64_t>(gridDim.x) * kWavesPerBlock;
  for (uint64_t seg = static_cast<uint64_t>(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6); seg < n_segs;
       seg += total_waves) {
    const uint64_t base = seg * kSegRows;
    uint64_t h[8];
    bool ok[8];
    load_hashes<K, DENSE>(a, base, n, lane, h, ok);
    uint64_t w[8], m[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      m[j] = mask_of(s_masks, h[j]);
      if constexpr (FILTER_IN_LDS) {
        w[j] = s_filter[block_of(h[j], block_mask)];
      } else {
        w[j] = ok[j] ? words[block_of(h[j], block_mask)] : 0ULL;
      }
    }
    uint64_t word[8];
    uint32_t cnt = 0;
    if constexpr (DENSE) {
      constexpr int V = KeyTraits<K>::kVec;
      uint64_t b[8];
#pragma unroll
      for (int j = 0; j < 8; j++) {
        b[j] = ballot64(ok[j] && (w[j] & m[j]) == m[j]);
        cnt += __popcll(b[j]);
      }
#pragma unroll
      for (int c = 0; c < 8 / V; c++) {
#pragma unroll
        for (int q = 0; q < V; q++) {
          uint64_t x = 0;
          if constexpr (V == 2) {
            x = spread2(b[c * 2 + 0] >> (32 * q)) | (spread2(b[c * 2 + 1] >> (32 * q)) << 1);
          } else {
#pragma unroll
            for (int e = 0; e < 4; e++) x |= spread4(b[c * 4 + e] >> (16 * q)) << e;
          }
          word[c * V + q] = x;
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; j++) {
        word[j] = ballot64(ok[j] && (w[j] & m[j]) == m[j]);
        cnt += __popcll(word[j]);
      }
    }
    uint64_t mine = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) mine = (lane == static_cast<uint32_t>(j)) ? word[j] : mine;
    if (lane < kWordsPerSeg) out_bits[seg * kWordsPerSeg + lane] = mine;
    if (seg_counts != nullptr && lane == 0) seg_counts[seg] = cnt;
  }
}

// ---- slice records -------------------------------------------------------------------------------
// A record carries the 30 hash bits a filter slice needs, laid out for the slice kernels' 32-bit ALU:
//   [0..4]   rotation & 31  (v_alignbit reads the low 5 bits of its shift operand: no extract)
//   [5..15]  index into the 2048-entry rotated-mask table: mask id (h & 1023) | rotation bit 5 << 10
//   [16..29] block within the slice ([30..31]: slice bits, masked off)
// Table entry (id, r5) = ROTL64(mask(id), 32 * r5). With r = 32 * r5 + t:
//   (w & ROTL(mask, r)) == ROTL(mask, r)  <=>  (ROTR(w, t) & entry) == entry
// and ROTR(w, t) for t < 32 is two v_alignbit_b32 — no 64-bit shifts, no rotation of the mask.
__device__ __forceinline__ uint32_t slice_record(uint64_t h) {
  const uint32_t x = static_cast<uint32_t>(h);
  return ((x >> kLogNumMasks) & 31u) | ((x & (kNumMasks - 1)) << 5) | (x & 0xFFFF8000u);
}
constexpr uint32_t kRotMasks = 2 * kNumMasks;
__device__ __forceinline__ void fill_rot_mask_table(uint64_t* s_rmasks) {
  for (int i = threadIdx.x; i < static_cast<int>(kRotMasks); i += blockDim.x) {
    const int id = i & (kNumMasks - 1), w = id >> 6, s = id & 63;
    const uint64_t lo = kMaskBits[w], hi = kMaskBits[w + 1];
    const uint64_t m = ((lo >> s) | ((hi << 1) << (63 - s))) & kFullMask;
    s_rmasks[i] = (i >> kLogNumMasks) ? rotl64(m, 32) : m;
  }
}
__device__ __forceinline__ uint64_t rot_entry(const uint64_t* s_rmasks, uint32_t rec) {
  return s_rmasks[(rec >> 5) & (kRotMasks - 1)];
}
__device__ __forceinline__ uint32_t rec_word(uint32_t rec) { return (rec >> 16) & (kSliceWords - 1); }
// the filter mask of a record: ROTL(entry, t)
__device__ __forceinline__ uint64_t rec_mask(const uint64_t* s_rmasks, uint32_t rec) {
  return rotl64(rot_entry(s_rmasks, rec), rec & 31u);
}
__device__ __forceinline__ bool probe_rec(const uint64_t* s_slice, const uint64_t* s_rmasks, uint32_t rec) {
  const uint64_t e = rot_entry(s_rmasks, rec);
  const uint64_t w = s_slice[rec_word(rec)];
  const uint32_t wl = static_cast<uint32_t>(w), wh = static_cast<uint32_t>(w >> 32);
  const uint32_t xl = __builtin_amdgcn_alignbit(wh, wl, rec), xh = __builtin_amdgcn_alignbit(wl, wh, rec);
  return ((~xl & static_cast<uint32_t>(e)) | (~xh & static_cast<uint32_t>(e >> 32))) == 0u;
}

// ---- partitioned probe, A: bucket a 16 Ki-row tile by filter slice --------------------------------
// Row r of the tile gets record slice_record(hash) stored at position pos(r) of the tile's
// slice-sorted record array (runs padded to kRunPad records); pos(r) is
// written per row (u16) so the unpermute step can restore row order. Per tile the padded runs
// (start << 16 | length) are written tile-major (one coalesced 4*P-byte row); runs_transpose_kernel
// turns them slice-major for the slice kernel. Two passes over the rows held in registers: count per
// slice (LDS atomics), scan, then claim positions with an LDS cursor per slice and scatter.
// Dynamic LDS: tile_cap record slots, then the per-slice count and cursor arrays.
template <int K, bool DENSE, bool MM>
__global__ __launch_bounds__(kTileThreads, RPT_PARTITION_MIN_WAVES) void partition_kernel(
    KeyArgs a, uint64_t n, uint32_t slice_mask, uint64_t n_tiles, uint32_t* __restrict__ recs,
    uint16_t* __restrict__ pos_out, uint32_t* __restrict__ runs_tm, int64_t* __restrict__ stats,
    const uint32_t* __restrict__ dev_n_tiles) {
  // dev_n_tiles (bucketed strategy): the tile count is only known on the device; the grid is an upper
  // bound and surplus workgroups leave (their run-table rows are never read).
  if (dev_n_tiles != nullptr && blockIdx.x >= *dev_n_tiles) return;
  extern __shared__ uint32_t s_dyn[];
  const uint64_t tile_cap = tile_cap_for(slice_mask + 1);
  uint32_t* s_rec = s_dyn;
  uint32_t* s_cnt = s_dyn + tile_cap;                  // rows per slice in this tile
  uint32_t* s_cur = s_dyn + tile_cap + slice_mask + 1;  // run start, then scatter cursor (start + count)
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t n_slices = slice_mask + 1;
  {  // one tile per workgroup (no persistent loop: keeps per-lane invariants out of registers)
    const uint64_t tile = blockIdx.x;
    for (uint32_t i = threadIdx.x; i < n_slices; i += kTileThreads) s_cnt[i] = 0;
    __syncthreads();
    const uint64_t tile_base = tile * kTileRows;
    // pass 1: hash, stage the record at its row position in LDS, count rows per slice; only the 16-bit
    // slice ids stay in registers (2 per word).
    static_assert(kMaxSliceCount <= 65536, "slice ids are packed as 16 bits");
    uint32_t sl2[kRowsPerThread / 2] = {};
    int64_t wmn = kMinInit, wmx = kMaxInit;  // wave-uniform: the key min/max stays out of VGPRs
#pragma unroll
    for (int sg = 0; sg < kSegsPerWaveA; sg++) {
      const uint32_t seg_local = wave * (kSegsPerWaveA * kSegRows) + sg * kSegRows;
      uint64_t hh[8];
      bool oo[8];
      int64_t mm[2] = {kMinInit, kMaxInit};
      load_hashes<K, DENSE, MM>(a, tile_base + seg_local, n, lane, hh, oo, mm);
      if constexpr (MM && K != kKeyHash) {
        wave_minmax(mm[0], mm[1]);
        wmn = min(wmn, mm[0]);
        wmx = max(wmx, mm[1]);
      }
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const uint32_t sl = static_cast<uint32_t>(hh[j] >> (kLogNumMasks + 6 + kSliceLog)) & slice_mask;
        s_rec[seg_local + seg_row<K, DENSE>(j, lane)] = slice_record(hh[j]);
        sl2[(sg * 8 + j) >> 1] |= sl << (16 * (j & 1));
        if (oo[j]) atomicAdd(&s_cnt[sl], 1u);
      }
    }
    if constexpr (MM && K != kKeyHash) publish_minmax(wmn, wmx, stats);
    __syncthreads();
    if (wave == 0) {  // exclusive scan of the slice counts, each padded to 4 records: kMaxSliceCount/64 per lane
      constexpr int kPer = kMaxSliceCount / 64;
      uint32_t c[kPer], t = 0;
#pragma unroll
      for (int i = 0; i < kPer; i++) {
        const uint32_t idx = lane * kPer + i;
        c[i] = idx < n_slices ? pad_run(s_cnt[idx]) : 0u;
        t += c[i];
      }
      uint32_t off = wave_inclusive_sum(t) - t;
#pragma unroll
      for (int i = 0; i < kPer; i++) {
        if (lane * kPer + i < n_slices) s_cur[lane * kPer + i] = off;
        off += c[i];
      }
    }
    // pass 2: pull this thread's records back out of the row-ordered staging ...
    uint32_t rec[kRowsPerThread];
#pragma unroll
    for (int sg = 0; sg < kSegsPerWaveA; sg++) {
      const uint32_t seg_local = wave * (kSegsPerWaveA * kSegRows) + sg * kSegRows;
#pragma unroll
      for (int j = 0; j < 8; j++) rec[sg * 8 + j] = s_rec[seg_local + seg_row<K, DENSE>(j, lane)];
    }
    __syncthreads();
    // ... and scatter them to their slice-sorted positions
#pragma unroll
    for (int sg = 0; sg < kSegsPerWaveA; sg++) {
      const uint64_t base = tile_base + wave * (kSegsPerWaveA * kSegRows) + sg * kSegRows;
      const uint32_t seg_rem = n > base ? static_cast<uint32_t>(n - base < kSegRows ? n - base : kSegRows) : 0u;
      uint16_t pv[8];
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const int jj = sg * 8 + j;
        const uint32_t sl = (sl2[jj >> 1] >> (16 * (jj & 1))) & 0xFFFFu;
        const bool ok = seg_row<K, DENSE>(j, lane) < seg_rem;
        uint32_t p = 0;
        if (ok) {
          p = atomicAdd(&s_cur[sl], 1u);
          s_rec[p] = rec[jj];
        }
        pv[j] = static_cast<uint16_t>(p);
      }
      // pos is padded to whole tiles: rows >= n get don't-care values. (nullptr: build, no row map)
      if (pos_out == nullptr) {
      } else if constexpr (DENSE) {
        constexpr int V = KeyTraits<K>::kVec;
#pragma unroll
        for (int c = 0; c < 8 / V; c++) {
          const uint64_t row0 = base + static_cast<uint64_t>(c) * 64 * V + static_cast<uint64_t>(lane) * V;
          if constexpr (V == 2) {
            *reinterpret_cast<uint32_t*>(pos_out + row0) =
                static_cast<uint32_t>(pv[c * 2]) | (static_cast<uint32_t>(pv[c * 2 + 1]) << 16);
          } else {
            *reinterpret_cast<uint64_t*>(pos_out + row0) =
                static_cast<uint64_t>(pv[c * 4]) | (static_cast<uint64_t>(pv[c * 4 + 1]) << 16) |
                (static_cast<uint64_t>(pv[c * 4 + 2]) << 32) | (static_cast<uint64_t>(pv[c * 4 + 3]) << 48);
          }
        }
      } else {
#pragma unroll
        for (int c = 0; c < 8; c++) pos_out[base + c * 64 + lane] = pv[c];
      }
    }
    __syncthreads();
    // records of the tile (pad slots hold stale values: probed, never read back); the scatter left
    // s_cur[i] = start_i + count_i
    const uint32_t used = s_cur[slice_mask] - s_cnt[slice_mask] + pad_run(s_cnt[slice_mask]);
    u32x4* dst = reinterpret_cast<u32x4*>(recs + tile * tile_cap);
    const u32x4* src = reinterpret_cast<const u32x4*>(s_rec);
    for (uint32_t i = threadIdx.x; i < used / 4; i += kTileThreads) dst[i] = src[i];
    for (uint32_t i = threadIdx.x; i < n_slices; i += kTileThreads)
      runs_tm[tile * n_slices + i] = ((s_cur[i] - s_cnt[i]) << 16) | s_cnt[i];  // start | true count
    __syncthreads();
  }
}

// runs_sm[slice][tile] = runs_tm[tile][slice], through 64 x 64 LDS tiles (both sides coalesced).
__global__ __launch_bounds__(kBlockThreads) void runs_transpose_kernel(const uint32_t* __restrict__ runs_tm,
                                                                      uint32_t n_slices, uint64_t n_tiles,
                                                                      uint32_t* __restrict__ runs_sm) {
  __shared__ uint32_t s_t[64][65];
  const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * 64;
  const uint32_t s0 = blockIdx.y * 64;
  const uint32_t c = threadIdx.x & 63, r0 = threadIdx.x >> 6;
  for (uint32_t r = r0; r < 64; r += 4) {
    const uint64_t t = t0 + r;
    s_t[r][c] = (t < n_tiles && s0 + c < n_slices) ? runs_tm[t * n_slices + s0 + c] : 0u;
  }
  __syncthreads();
  for (uint32_t r = r0; r < 64; r += 4) {
    const uint64_t t = t0 + c;
    if (t < n_tiles && s0 + r < n_slices) runs_sm[static_cast<uint64_t>(s0 + r) * n_tiles + t] = s_t[c][r];
  }
}

// ---- partitioned probe, B: one workgroup per (slice, tile range) probes its records from LDS -------

// The runs of 64 consecutive tiles are walked as ONE flattened record stream per wave: record k of
// the stream belongs to the tile whose inclusive run-length prefix first exceeds k. Runs are padded
// to kRunPad = 8 records, so each lane owns 8 consecutive, 32-byte aligned records of one run: two
// 16-B loads and one byte of pass bits per lane, 512 records per wave step. The (uniform) tile cursor
// lives in scalar registers; a step visits only the few tiles its 512 records overlap. Record offsets
// are 32-bit relative to the batch's first tile (a uniform base pointer).
// Which tiles and run-table row a slice workgroup walks. Plain partitioned: all n_tiles tiles, run row
// = slice. Bucketed (bucket_tiles != nullptr): global slice g = bucket * kBucketSlices + local slice;
// the bucket's tiles are [bucket_tiles[b], bucket_tiles[b+1]) and the run row is the local slice.
struct SliceWork {
  uint32_t slice, run_row;
  uint64_t t_lo, t_hi;
};
__device__ __forceinline__ SliceWork slice_work(uint32_t item, uint32_t splits, uint64_t n_tiles,
                                                const uint32_t* bucket_tiles) {
  const uint32_t slice = item / splits, part = item % splits;
  uint64_t lo = 0, cnt = n_tiles;
  uint32_t row = slice;
  if (bucket_tiles != nullptr) {
    const uint32_t b = slice >> kBucketSliceLog;
    lo = bucket_tiles[b];
    cnt = bucket_tiles[b + 1] - lo;
    row = slice & (kBucketSlices - 1);
  }
  return SliceWork{slice, row, lo + cnt * part / splits, lo + cnt * (part + 1) / splits};
}

// Probe the runs of tiles [sw.t_lo, sw.t_hi) of one slice held in LDS (see above).
// Tiles per wave batch: 64 (one run per lane), or fewer so that all kSliceThreads/64 waves get work.
__device__ __forceinline__ uint32_t batch_tiles(uint64_t n_t) {
  constexpr uint64_t kWaves = kSliceThreads / 64;
  return static_cast<uint32_t>(n_t >= 64 * kWaves ? 64 : (n_t + kWaves - 1) / kWaves);
}

__device__ __forceinline__ void probe_slice_runs(const uint64_t* s_slice, const uint64_t* s_rmasks, const SliceWork& sw,
                                                 uint64_t n_tiles, const uint32_t* __restrict__ recs,
                                                 const uint32_t* __restrict__ runs, uint8_t* __restrict__ passbits,
                                                 uint32_t tile_cap) {
  constexpr int kUnroll = RPT_SLICE_UNROLL;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr uint32_t kWaves = kSliceThreads / 64;
  const uint64_t t_lo = sw.t_lo, t_hi = sw.t_hi;
  const uint32_t* my_runs = runs + static_cast<uint64_t>(sw.run_row) * n_tiles;
  // a wave walks batches of bt <= 64 consecutive tiles (one run per lane); few tiles per slice (the
  // bucketed strategy) are spread over all waves in smaller batches
  const uint32_t bt = batch_tiles(t_hi - t_lo);
  const uint32_t my = lane < bt ? lane : ~0u >> 1;  // lanes >= bt hold no run
  uint32_t info_next = (t_lo + wave * bt + my < t_hi) ? my_runs[t_lo + wave * bt + my] : 0u;
  for (uint64_t tb = t_lo + wave * bt; tb < t_hi; tb += kWaves * bt) {
    const uint32_t info = info_next;  // the next batch's runs are fetched while this one is probed
    info_next = (tb + kWaves * bt + my < t_hi) ? my_runs[tb + kWaves * bt + my] : 0u;
    const uint32_t cnt = pad_run(info & 0xFFFFu);  // padded run length (multiple of kRunPad)
    const uint32_t start = lane * tile_cap + (info >> 16);
    const uint32_t* brecs = recs + tb * tile_cap;  // uniform
    uint8_t* bpass = passbits + tb * (tile_cap / kRunPad);
    const uint32_t incl = wave_inclusive_sum(cnt);
    const uint32_t total = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), 63));
    uint32_t j = 0;  // uniform: first tile of the batch whose inclusive prefix exceeds the step start
    constexpr uint32_t kStep = 64 * kRunPad;  // records per wave step
    for (uint32_t k0 = 0; k0 < total; k0 += kStep * kUnroll) {
      uint32_t off[kUnroll];
      u32x4 rec[kUnroll][2];
#pragma unroll
      for (int u = 0; u < kUnroll; u++) {
        const uint32_t kf = k0 + u * kStep;
        const uint32_t k = kf + lane * kRunPad;
        off[u] = ~0u;
        if (kf < total) {
          while (static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), j)) <= kf) j++;
          const uint32_t kl = (kf + kStep - 1 < total) ? kf + kStep - 1 : total - 1;
          for (uint32_t jj = j;; jj++) {
            const uint32_t inc = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), jj));
            const uint32_t c = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(cnt), jj));
            const uint32_t b = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(start), jj));
            if (k >= inc - c && k < inc) off[u] = b + (k - (inc - c));
            if (inc > kl) break;
          }
        }
        rec[u][0] = rec[u][1] = u32x4{0, 0, 0, 0};
        if (off[u] != ~0u) {
          rec[u][0] = *reinterpret_cast<const u32x4*>(brecs + off[u]);
          rec[u][1] = *reinterpret_cast<const u32x4*>(brecs + off[u] + 4);
        }
      }
#pragma unroll
      for (int u = 0; u < kUnroll; u++) {
        uint32_t bits = 0;
#pragma unroll
        for (int e = 0; e < 8; e++) bits |= static_cast<uint32_t>(probe_rec(s_slice, s_rmasks, rec[u][e >> 2][e & 3])) << e;
        if (off[u] != ~0u) bpass[off[u] / kRunPad] = static_cast<uint8_t>(bits);
      }
    }
  }
}

// First work item >= item (stepping by gridDim.x) that has tiles; n_items if none.
__device__ __forceinline__ uint32_t next_item(uint32_t item, uint32_t n_items, uint32_t splits, uint64_t n_tiles,
                                              const uint32_t* bucket_tiles, SliceWork& sw) {
  for (; item < n_items; item += gridDim.x) {
    sw = slice_work(item, splits, n_tiles, bucket_tiles);
    if (sw.t_lo < sw.t_hi) break;
  }
  return item;
}

// Work items (slice, split) are walked by a resident grid; when a workgroup has several (filters with
// more slices than the chip has CUs: the bucketed strategy), the next item's slice is fetched into
// registers (128 B per thread) while the current one is probed, then stored to LDS.
__global__ __launch_bounds__(kSliceThreads) void slice_probe_kernel(const uint64_t* __restrict__ words,
                                                                   uint32_t splits, uint64_t n_tiles,
                                                                   const uint32_t* __restrict__ recs,
                                                                   const uint32_t* __restrict__ runs,
                                                                   uint8_t* __restrict__ passbits,
                                                                   uint32_t tile_slices,
                                                                   const uint32_t* __restrict__ bucket_tiles,
                                                                   uint32_t n_items) {
  // one LDS array, table first: the slice's base offset folds into the ds_read immediate
  __shared__ uint64_t s_lds[kRotMasks + kSliceWords];
  uint64_t* const s_rmasks = s_lds;
  uint64_t* const s_slice = s_lds + kRotMasks;
  u64x2* const s_slice2 = reinterpret_cast<u64x2*>(s_slice);
  constexpr uint32_t kPre = kSliceWords / 2 / kSliceThreads;  // 16-B pieces of a slice per thread
  SliceWork cur;
  uint32_t item = next_item(blockIdx.x, n_items, splits, n_tiles, bucket_tiles, cur);
  if (item >= n_items) return;  // uniform
  {
    const u64x2* src = reinterpret_cast<const u64x2*>(words + static_cast<uint64_t>(cur.slice) * kSliceWords);
#pragma unroll
    for (uint32_t i = 0; i < kPre; i++) s_slice2[threadIdx.x + i * kSliceThreads] = src[threadIdx.x + i * kSliceThreads];
  }
  fill_rot_mask_table(s_rmasks);
  const uint32_t tile_cap = static_cast<uint32_t>(tile_cap_for(tile_slices));
  while (true) {
    __syncthreads();
    SliceWork nxt;
    const uint32_t nitem = next_item(item + gridDim.x, n_items, splits, n_tiles, bucket_tiles, nxt);
    u64x2 pre[kPre];
    if (nitem < n_items) {
      const u64x2* src = reinterpret_cast<const u64x2*>(words + static_cast<uint64_t>(nxt.slice) * kSliceWords);
#pragma unroll
      for (uint32_t i = 0; i < kPre; i++) pre[i] = src[threadIdx.x + i * kSliceThreads];
    }
    probe_slice_runs(s_slice, s_rmasks, cur, n_tiles, recs, runs, passbits, tile_cap);
    if (nitem >= n_items) break;
    __syncthreads();  // every wave is done with this slice
#pragma unroll
    for (uint32_t i = 0; i < kPre; i++) s_slice2[threadIdx.x + i * kSliceThreads] = pre[i];
    item = nitem;
    cur = nxt;
  }
}

// ---- partitioned build: OR each slice's records into an LDS copy, then merge into the filter ----
// Same flattened run walk as slice_probe_kernel. The slice starts from zero in LDS (ds_or_b64 per
// record) and is merged into the filter with coalesced 64-bit device-scope atomic ORs of its non-zero
// words, so concurrent inserts and several workgroups per slice compose (OR is idempotent).
__global__ __launch_bounds__(kSliceThreads) void slice_insert_kernel(uint64_t* __restrict__ words, uint32_t splits,
                                                                    uint64_t n_tiles,
                                                                    const uint32_t* __restrict__ recs,
                                                                    const uint32_t* __restrict__ runs,
                                                                    uint32_t tile_slices,
                                                                    const uint32_t* __restrict__ bucket_tiles) {
  // one LDS array, table first: the slice's base offset folds into the ds_read immediate
  __shared__ uint64_t s_lds[kRotMasks + kSliceWords];
  uint64_t* const s_rmasks = s_lds;
  uint64_t* const s_slice = s_lds + kRotMasks;
  const SliceWork sw = slice_work(blockIdx.x, splits, n_tiles, bucket_tiles);
  const uint32_t slice = sw.slice;
  const uint64_t t_lo = sw.t_lo, t_hi = sw.t_hi;
  if (t_lo >= t_hi) return;  // no rows reach this slice (uniform)
  for (uint32_t i = threadIdx.x; i < kSliceWords; i += kSliceThreads) s_slice[i] = 0;
  fill_rot_mask_table(s_rmasks);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr uint32_t kWaves = kSliceThreads / 64;
  const uint32_t* my_runs = runs + static_cast<uint64_t>(sw.run_row) * n_tiles;
  const uint64_t tile_cap = tile_cap_for(tile_slices);
  const uint32_t bt = batch_tiles(t_hi - t_lo);  // as slice_probe_kernel
  for (uint64_t tb = t_lo + wave * bt; tb < t_hi; tb += kWaves * bt) {
    const uint32_t info = (lane < bt && tb + lane < t_hi) ? my_runs[tb + lane] : 0u;
    const uint32_t real = info & 0xFFFFu;      // records of the run
    const uint32_t cnt = pad_run(real);          // padded length (k-space)
    const uint64_t base = (tb + lane) * tile_cap + (info >> 16);
    const uint32_t base_lo = static_cast<uint32_t>(base), base_hi = static_cast<uint32_t>(base >> 32);
    const uint32_t incl = wave_inclusive_sum(cnt);
    const uint32_t total = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), 63));
    uint32_t j = 0;
    constexpr uint32_t kStep = 64 * kRunPad;
    for (uint32_t kf = 0; kf < total; kf += kStep) {
      const uint32_t k = kf + lane * kRunPad;
      while (static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), j)) <= kf) j++;
      const uint32_t kl = (kf + kStep - 1 < total) ? kf + kStep - 1 : total - 1;
      uint64_t addr = ~0ULL;
      uint32_t nreal = 0;  // how many of this lane's kRunPad slots are real records (pad slots are stale)
      for (uint32_t jj = j;; jj++) {
        const uint32_t inc = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), jj));
        const uint32_t c = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(cnt), jj));
        const uint32_t rl = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(real), jj));
        const uint64_t b =
            static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(base_lo), jj))) |
            (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(base_hi), jj))) << 32);
        if (k >= inc - c && k < inc) {
          const uint32_t off = k - (inc - c);
          addr = b + off;
          nreal = rl > off ? (rl - off < kRunPad ? rl - off : kRunPad) : 0;
        }
        if (inc > kl) break;
      }
      if (addr != ~0ULL) {
        const u32x4 r0 = *reinterpret_cast<const u32x4*>(recs + addr);
        const u32x4 r1 = *reinterpret_cast<const u32x4*>(recs + addr + 4);
#pragma unroll
        for (uint32_t e = 0; e < kRunPad; e++) {
          if (e < nreal) {
            const uint32_t rec = e < 4 ? r0[e] : r1[e - 4];
            atomicOr(reinterpret_cast<unsigned long long*>(&s_slice[rec_word(rec)]),
                     static_cast<unsigned long long>(rec_mask(s_rmasks, rec)));
          }
        }
      }
    }
  }
  __syncthreads();
  uint64_t* dst = words + static_cast<uint64_t>(slice) * kSliceWords;
  for (uint32_t i = threadIdx.x; i < kSliceWords; i += kSliceThreads) {
    const uint64_t v = s_slice[i];
    if (v) __hip_atomic_fetch_or(dst + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---- partitioned probe, C: restore row order -> result bits + per-segment counts (P1's format) -----
// One 256-thread workgroup per tile: the tile's pass bits (tile_cap / 8 bytes) are staged in LDS while
// each wave's row positions are already in flight; a lane owns 8 consecutive rows of a segment (one
// 16-B load of positions) and produces byte `lane` of the segment's 512-bit row-ordered result.
constexpr int kUnpermuteThreads = 256;
__global__ __launch_bounds__(kUnpermuteThreads) void unpermute_kernel(const uint16_t* __restrict__ pos,
                                                                     const uint8_t* __restrict__ passbits, uint64_t n,
                                                                     uint64_t tile_cap,
                                                                     uint64_t* __restrict__ out_bits,
                                                                     uint32_t* __restrict__ seg_counts,
                                                                     const uint32_t* __restrict__ dev_n_tiles) {
  if (dev_n_tiles != nullptr && blockIdx.x >= *dev_n_tiles) return;  // bucketed: grid is an upper bound
  extern __shared__ uint8_t s_pass[];  // tile_cap / 8 bytes of pass bits (record order)
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t n_segs = (n + kSegRows - 1) / kSegRows;
  constexpr uint32_t kSegsPerWave = (kTileRows / kSegRows) / (kUnpermuteThreads / 64);
  const uint64_t tile = blockIdx.x;
  const uint64_t seg0 = tile * (kTileRows / kSegRows) + wave * kSegsPerWave;
  u32x4 pv[kSegsPerWave];  // 8 row positions (u16) per lane per segment
#pragma unroll
  for (uint32_t sg = 0; sg < kSegsPerWave; sg++) {
    pv[sg] = u32x4{0, 0, 0, 0};
    if (seg0 + sg < n_segs) pv[sg] = *reinterpret_cast<const u32x4*>(pos + (seg0 + sg) * kSegRows + lane * 8);
  }
  {
    const u32x4* src = reinterpret_cast<const u32x4*>(passbits + tile * (tile_cap / 8));
    for (uint32_t i = threadIdx.x; i < tile_cap / 128; i += kUnpermuteThreads) reinterpret_cast<u32x4*>(s_pass)[i] = src[i];
  }
  __syncthreads();
  uint8_t* out_bytes = reinterpret_cast<uint8_t*>(out_bits);
#pragma unroll
  for (uint32_t sg = 0; sg < kSegsPerWave; sg++) {
    const uint64_t seg = seg0 + sg;
    if (seg >= n_segs) break;
    uint32_t byte = 0;
#pragma unroll
    for (int e = 0; e < 8; e++) {
      const uint32_t p = (pv[sg][e >> 1] >> (16 * (e & 1))) & 0xFFFFu;
      byte |= ((static_cast<uint32_t>(s_pass[p >> 3]) >> (p & 7)) & 1u) << e;
    }
    const uint64_t row0 = seg * kSegRows + lane * 8;  // rows >= n (last segment) carry don't-care positions
    if (row0 + 8 > n) byte = row0 >= n ? 0u : byte & ((1u << (n - row0)) - 1u);
    out_bytes[seg * (kSegRows / 8) + lane] = static_cast<uint8_t>(byte);
    if (seg_counts != nullptr) {
      const uint32_t cnt = wave_sum(__popc(byte));
      if (lane == 0) seg_counts[seg] = cnt;
    }
  }
}

// ---- bucketed strategy (filters of 2^22..2^31 blocks) ----------------------------------------------
// Level 1 cuts the rows by 16 MiB filter region ("bucket": 128 slices) into one contiguous hash array
// per bucket, each padded to whole 16 Ki-row tiles; level 2 is the partitioned pipeline above over
// those arrays, every bucket against its own 128 slices. bucket = block id >> 21 = hash bits 37...
__device__ __forceinline__ uint32_t bucket_of(uint64_t h, uint32_t bucket_mask) {
  return static_cast<uint32_t>(h >> (kLogNumMasks + 6 + kSliceLog + kBucketSliceLog)) & bucket_mask;
}

// B1: rows per bucket of every 16 Ki-row level-1 tile -> counts_tm[tile][bucket] (+ the build's min/max).
template <int K, bool DENSE, bool MM>
__global__ __launch_bounds__(kTileThreads) void bucket_count_kernel(KeyArgs a, uint64_t n, uint32_t bucket_mask,
                                                                    uint32_t* __restrict__ counts_tm,
                                                                    int64_t* __restrict__ stats) {
  __shared__ uint32_t s_cnt[kMaxBuckets];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t nb = bucket_mask + 1;
  for (uint32_t i = threadIdx.x; i < nb; i += kTileThreads) s_cnt[i] = 0;
  __syncthreads();
  const uint64_t tile = blockIdx.x, tile_base = tile * kTileRows;
  int64_t wmn = kMinInit, wmx = kMaxInit;
#pragma unroll
  for (int sg = 0; sg < kSegsPerWaveA; sg++) {
    const uint32_t seg_local = wave * (kSegsPerWaveA * kSegRows) + sg * kSegRows;
    uint64_t hh[8];
    bool oo[8];
    int64_t mm[2] = {kMinInit, kMaxInit};
    load_hashes<K, DENSE, MM>(a, tile_base + seg_local, n, lane, hh, oo, mm);
    if constexpr (MM && K != kKeyHash) {
      wave_minmax(mm[0], mm[1]);
      wmn = min(wmn, mm[0]);
      wmx = max(wmx, mm[1]);
    }
#pragma unroll
    for (int j = 0; j < 8; j++)
      if (oo[j]) atomicAdd(&s_cnt[bucket_of(hh[j], bucket_mask)], 1u);
  }
  if constexpr (MM && K != kKeyHash) publish_minmax(wmn, wmx, stats);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nb; i += kTileThreads) counts_tm[tile * nb + i] = s_cnt[i];
}

// B2: in place, each bucket's row of counts_bm[bucket][tile] becomes its exclusive prefix over tiles
// (where the tile's run starts inside the bucket's array); totals[bucket] = the bucket's rows.
__global__ __launch_bounds__(1024) void bucket_scan_kernel(uint32_t* __restrict__ counts_bm, uint64_t n_tiles,
                                                          uint32_t* __restrict__ totals) {
  __shared__ uint32_t s_wave[16];
  uint32_t* row = counts_bm + static_cast<uint64_t>(blockIdx.x) * n_tiles;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t carry = 0;
  for (uint64_t c0 = 0; c0 < n_tiles; c0 += 1024) {
    const uint64_t i = c0 + threadIdx.x;
    const uint32_t v = i < n_tiles ? row[i] : 0u;
    const uint32_t incl = wave_inclusive_sum(v);
    if (lane == 63) s_wave[wave] = incl;
    __syncthreads();
    uint32_t off = carry, chunk = 0;
    for (uint32_t w = 0; w < 16; w++) {
      const uint32_t t = s_wave[w];
      off += w < wave ? t : 0u;
      chunk += t;
    }
    if (i < n_tiles) row[i] = off + incl - v;
    carry += chunk;
    __syncthreads();
  }
  if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

// B3: bucket bases in the level-2 array (each bucket padded to whole tiles) and its tile ranges:
// base[b] (rows), bucket_tiles[b] = base[b] / kTileRows; base[nb], bucket_tiles[nb] = the totals.
__global__ __launch_bounds__(1024) void bucket_base_kernel(const uint32_t* __restrict__ totals, uint32_t nb,
                                                          uint64_t* __restrict__ base,
                                                          uint32_t* __restrict__ bucket_tiles) {
  __shared__ uint32_t s_wave[16];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t b = threadIdx.x;
  const uint32_t tiles = b < nb ? static_cast<uint32_t>((totals[b] + kTileRows - 1) / kTileRows) : 0u;
  const uint32_t incl = wave_inclusive_sum(tiles);
  if (lane == 63) s_wave[wave] = incl;
  __syncthreads();
  uint32_t off = 0, all = 0;
  for (uint32_t w = 0; w < 16; w++) {
    off += w < wave ? s_wave[w] : 0u;
    all += s_wave[w];
  }
  const uint32_t first = off + incl - tiles;
  if (b < nb) {
    bucket_tiles[b] = first;
    base[b] = static_cast<uint64_t>(first) * kTileRows;
  }
  if (b == 0) {
    bucket_tiles[nb] = all;
    base[nb] = static_cast<uint64_t>(all) * kTileRows;
  }
}

// B4: hash every row of a level-1 tile again, sort the tile's hashes by bucket in LDS and copy each
// bucket's run to its place in that bucket's array: hashes[base[b] + pre_tm[tile][b] + i]. pos_out (u16,
// probe only) records each row's position in the tile's bucket-sorted order.
template <int K, bool DENSE>
__global__ __launch_bounds__(kTileThreads) void bucket_scatter_kernel(KeyArgs a, uint64_t n, uint32_t bucket_mask,
                                                                      const uint32_t* __restrict__ counts_tm,
                                                                      const uint32_t* __restrict__ pre_tm,
                                                                      const uint64_t* __restrict__ base,
                                                                      uint64_t* __restrict__ hashes,
                                                                      uint16_t* __restrict__ pos_out) {
  extern __shared__ uint64_t s_h[];  // kTileRows hashes, bucket-sorted
  __shared__ uint32_t s_start[kMaxBuckets], s_cur[kMaxBuckets];
  __shared__ uint64_t s_dst[kMaxBuckets];  // where each bucket's run goes in the level-2 array
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t nb = bucket_mask + 1;
  // Workgroups go round-robin to the 8 XCDs; give each XCD a contiguous range of tiles, so the runs of
  // neighbouring tiles (adjacent in each bucket's array) are written through the same L2 and leave it
  // as whole lines.
  const uint32_t per_xcd = gridDim.x / 8, xcd = blockIdx.x % 8;
  const uint64_t tile = blockIdx.x < per_xcd * 8 ? static_cast<uint64_t>(xcd) * per_xcd + blockIdx.x / 8 : blockIdx.x;
  const uint64_t tile_base = tile * kTileRows;
  const uint32_t* cnt = counts_tm + tile * nb;
  for (uint32_t i = threadIdx.x; i < nb; i += kTileThreads) s_dst[i] = base[i] + pre_tm[tile * nb + i];
  if (wave == 0) {  // exclusive scan of this tile's bucket counts, kMaxBuckets / 64 per lane
    constexpr int kPer = kMaxBuckets / 64;
    uint32_t c[kPer], t = 0;
#pragma unroll
    for (int i = 0; i < kPer; i++) {
      const uint32_t idx = lane * kPer + i;
      c[i] = idx < nb ? cnt[idx] : 0u;
      t += c[i];
    }
    uint32_t off = wave_inclusive_sum(t) - t;
#pragma unroll
    for (int i = 0; i < kPer; i++) {
      const uint32_t idx = lane * kPer + i;
      if (idx < nb) s_start[idx] = s_cur[idx] = off;
      off += c[i];
    }
  }
  __syncthreads();
#pragma unroll
  for (int sg = 0; sg < kSegsPerWaveA; sg++) {
    const uint32_t seg_local = wave * (kSegsPerWaveA * kSegRows) + sg * kSegRows;
    const uint64_t sbase = tile_base + seg_local;
    uint64_t hh[8];
    bool oo[8];
    load_hashes<K, DENSE>(a, sbase, n, lane, hh, oo);
    uint16_t pv[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint32_t p = 0;
      if (oo[j]) {
        p = atomicAdd(&s_cur[bucket_of(hh[j], bucket_mask)], 1u);
        s_h[p] = hh[j];
      }
      pv[j] = static_cast<uint16_t>(p);
    }
    if (pos_out != nullptr) {  // padded to whole tiles: rows >= n get don't-care values
#pragma unroll
      for (int j = 0; j < 8; j++) pos_out[sbase + seg_row<K, DENSE>(j, lane)] = pv[j];
    }
  }
  __syncthreads();
  for (uint32_t b = wave; b < nb; b += kTileThreads / 64) {  // LDS only: no global latency in the chain
    const uint32_t c = s_cur[b] - s_start[b];
    uint64_t* dst = hashes + s_dst[b];
    const uint64_t* src = s_h + s_start[b];
    for (uint32_t i = lane; i < c; i += 64) dst[i] = src[i];
  }
}

// B5: pad each bucket's array to whole tiles with copies of its first hash (re-inserting or re-probing
// a present hash changes nothing, and the pads' results are never read).
__global__ __launch_bounds__(kBlockThreads) void bucket_pad_kernel(const uint32_t* __restrict__ totals,
                                                                  const uint64_t* __restrict__ base,
                                                                  uint64_t* __restrict__ hashes) {
  const uint32_t b = blockIdx.x;
  const uint64_t t = totals[b], b0 = base[b], end = base[b + 1];
  if (t == 0) return;
  const uint64_t v = hashes[b0];
  for (uint64_t i = b0 + t + threadIdx.x; i < end; i += kBlockThreads) hashes[i] = v;
}

// B6: level-1 unpermute. Per level-1 tile: gather the pass bits of its bucket runs out of the level-2
// result bits (bits2, level-2 array order) into LDS in the tile's bucket-sorted order, 64-bit pieces
// per item (run, piece), then map every row through its position (pos1) -> result bits + counts.
constexpr int kBucketUnpermuteThreads = 256;
__global__ __launch_bounds__(kBucketUnpermuteThreads) void bucket_unpermute_kernel(
    const uint16_t* __restrict__ pos1, const uint64_t* __restrict__ bits2, uint64_t n, uint32_t bucket_mask,
    const uint32_t* __restrict__ counts_tm, const uint32_t* __restrict__ pre_tm, const uint64_t* __restrict__ base,
    uint64_t* __restrict__ out_bits, uint32_t* __restrict__ seg_counts) {
  __shared__ uint32_t s_bits[kTileRows / 32];
  __shared__ uint32_t s_start[kMaxBuckets], s_item[kMaxBuckets + 1], s_cnt[kMaxBuckets];
  __shared__ uint64_t s_g[kMaxBuckets];
  __shared__ uint32_t s_wave[kBucketUnpermuteThreads / 64][2];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr uint32_t kWaves = kBucketUnpermuteThreads / 64;
  const uint32_t nb = bucket_mask + 1;
  const uint64_t tile = blockIdx.x;
  const uint64_t n_segs = (n + kSegRows - 1) / kSegRows;
  constexpr uint32_t kSegsPerWave = (kTileRows / kSegRows) / kWaves;
  const uint64_t seg0 = tile * (kTileRows / kSegRows) + wave * kSegsPerWave;
  u32x4 pv[kSegsPerWave];  // row positions, in flight while the bits are staged
#pragma unroll
  for (uint32_t sg = 0; sg < kSegsPerWave; sg++) {
    pv[sg] = u32x4{0, 0, 0, 0};
    if (seg0 + sg < n_segs) pv[sg] = *reinterpret_cast<const u32x4*>(pos1 + (seg0 + sg) * kSegRows + lane * 8);
  }
  for (uint32_t i = threadIdx.x; i < kTileRows / 32; i += kBucketUnpermuteThreads) s_bits[i] = 0;
  // per bucket: run length, start in the tile's sorted order, start in bits2, 64-bit pieces (scans by
  // the whole workgroup, kMaxBuckets / 256 buckets per thread)
  constexpr int kPer = kMaxBuckets / kBucketUnpermuteThreads;
  uint32_t c[kPer], k[kPer], tc = 0, tk = 0;
#pragma unroll
  for (int i = 0; i < kPer; i++) {
    const uint32_t b = threadIdx.x * kPer + i;
    c[i] = b < nb ? counts_tm[tile * nb + b] : 0u;
    k[i] = (c[i] + 63) / 64;
    tc += c[i];
    tk += k[i];
    if (b < nb) {
      s_cnt[b] = c[i];
      s_g[b] = base[b] + pre_tm[tile * nb + b];
    }
  }
  const uint32_t ic = wave_inclusive_sum(tc), ik = wave_inclusive_sum(tk);
  if (lane == 63) {
    s_wave[wave][0] = ic;
    s_wave[wave][1] = ik;
  }
  __syncthreads();
  uint32_t oc = ic - tc, ok_ = ik - tk, total_items = 0;
  for (uint32_t w = 0; w < kWaves; w++) {
    oc += w < wave ? s_wave[w][0] : 0u;
    ok_ += w < wave ? s_wave[w][1] : 0u;
    total_items += s_wave[w][1];
  }
#pragma unroll
  for (int i = 0; i < kPer; i++) {
    const uint32_t b = threadIdx.x * kPer + i;
    if (b < nb) {
      s_start[b] = oc;
      s_item[b] = ok_;
    }
    oc += c[i];
    ok_ += k[i];
  }
  if (threadIdx.x == 0) s_item[nb] = total_items;
  __syncthreads();
  for (uint32_t it = threadIdx.x; it < total_items; it += kBucketUnpermuteThreads) {
    uint32_t lo = 0, hi = nb;  // last bucket whose first item <= it
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (s_item[mid] <= it) lo = mid;
      else hi = mid;
    }
    const uint32_t b = lo, piece = it - s_item[b];
    const uint32_t len = min(64u, s_cnt[b] - piece * 64);
    const uint64_t q = s_g[b] + piece * 64ULL;
    const uint32_t sh = static_cast<uint32_t>(q & 63);
    const uint64_t w0 = bits2[q >> 6];
    uint64_t v = w0 >> sh;
    if (sh != 0 && sh + len > 64) v |= bits2[(q >> 6) + 1] << (64 - sh);
    if (len < 64) v &= (1ULL << len) - 1;
    const uint32_t d = s_start[b] + piece * 64;  // destination bit in the tile's sorted order
    const uint32_t dw = d >> 5, ds = d & 31;
    atomicOr(&s_bits[dw], static_cast<uint32_t>(v << ds));
    if (len + ds > 32) atomicOr(&s_bits[dw + 1], static_cast<uint32_t>(v >> (32 - ds)));
    if (len + ds > 64) atomicOr(&s_bits[dw + 2], static_cast<uint32_t>(v >> (64 - ds)));
  }
  __syncthreads();
  uint8_t* out_bytes = reinterpret_cast<uint8_t*>(out_bits);
#pragma unroll
  for (uint32_t sg = 0; sg < kSegsPerWave; sg++) {
    const uint64_t seg = seg0 + sg;
    if (seg >= n_segs) break;
    uint32_t byte = 0;
#pragma unroll
    for (int e = 0; e < 8; e++) {
      const uint32_t p = (pv[sg][e >> 1] >> (16 * (e & 1))) & 0xFFFFu;
      byte |= ((s_bits[p >> 5] >> (p & 31)) & 1u) << e;
    }
    const uint64_t row0 = seg * kSegRows + lane * 8;
    if (row0 + 8 > n) byte = row0 >= n ? 0u : byte & ((1u << (n - row0)) - 1u);
    out_bytes[seg * (kSegRows / 8) + lane] = static_cast<uint8_t>(byte);
    const uint32_t cnt = wave_sum(__popc(byte));
    if (lane == 0) seg_counts[seg] = cnt;
  }
}

// ---- P2a: survivor count per group of 1024 segments --------------------------------------------
__global__ __launch_bounds__(kBlockThreads) void group_sum_kernel(const uint32_t* __restrict__ seg_counts,
                                                                 uint64_t n_segs, uint32_t* __restrict__ group_sums) {
  static_assert(kGroupSegs == kBlockThreads, "one segment count per thread");
  __shared__ uint32_t s_part[kWavesPerBlock];
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kGroupSegs + threadIdx.x;
  uint32_t s = i < n_segs ? seg_counts[i] : 0u;
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) group_sums[blockIdx.x] = s_part[0] + s_part[1] + s_part[2] + s_part[3];
}

// ---- P2b: exclusive scan of the group sums (one 1024-thread workgroup; <= 8192 groups) ----------
__global__ __launch_bounds__(1024) void group_scan_kernel(const uint32_t* __restrict__ group_sums, uint32_t n_groups,
                                                         uint32_t* __restrict__ group_offs,
                                                         uint64_t* __restrict__ out_count) {
  __shared__ uint32_t s_wave[16];
  const uint32_t per = (n_groups + 1023) / 1024;
  const uint32_t first = threadIdx.x * per;
  uint32_t local = 0;
  for (uint32_t i = first; i < first + per && i < n_groups; i++) local += group_sums[i];
  const uint32_t incl = wave_inclusive_sum(local);
  const uint32_t wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 63) s_wave[wave] = incl;
  __syncthreads();
  uint32_t wave_off = 0;
  for (uint32_t w = 0; w < wave; w++) wave_off += s_wave[w];
  uint32_t run = wave_off + incl - local;
  for (uint32_t i = first; i < first + per && i < n_groups; i++) {
    group_offs[i] = run;
    run += group_sums[i];
  }
  if (threadIdx.x == 1023) {
    uint32_t total = 0;
    for (int w = 0; w < 16; w++) total += s_wave[w];
    *out_count = total;
  }
}

// ---- P3: expand result bits into an ascending selection vector ----------------------------------
__global__ __launch_bounds__(kBlockThreads) void compact_kernel(const uint64_t* __restrict__ bits,
                                                               const uint32_t* __restrict__ seg_counts, uint64_t n_segs,
                                                               const uint32_t* __restrict__ group_offs,
                                                               const uint32_t* __restrict__ row_sel,
                                                               uint32_t* __restrict__ out_sel) {
  __shared__ uint32_t s_off[kGroupSegs];
  __shared__ uint32_t s_wave[kWavesPerBlock];
  __shared__ uint16_t s_stage[kWavesPerBlock][8 * kSegRows];  // one 4096-row step per wave (row offsets)
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
  // Each wave expands 8 segments (64 words = 4096 rows) per step: survivors are first written to the
  // wave's LDS buffer in row order, then streamed out with coalesced stores.
  uint16_t* buf = s_stage[wave];
  constexpr uint32_t kSteps = kGroupSegs / 8 / kWavesPerBlock;
  uint64_t words[kSteps];  // all of this wave's result words in flight at once
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
    uint64_t word = words[i];
    const uint32_t pc = __popcll(word);
    const uint32_t incl = wave_inclusive_sum(pc);
    const uint32_t total = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), 63));
    uint32_t p = incl - pc;
    while (word) {
      buf[p++] = static_cast<uint16_t>(lane * 64 + __builtin_ctzll(word));
      word &= word - 1;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    uint32_t* dst = out_sel + s_off[b * 8];
    const uint32_t step_row = static_cast<uint32_t>(seg0 * kSegRows);
    for (uint32_t q = lane; q < total; q += 64) {
      const uint32_t row = step_row + buf[q];
      dst[q] = row_sel ? row_sel[row] : row;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ---- k2: insert ----------------------------------------------------------------------------------
template <int K, bool DENSE>
__global__ __launch_bounds__(kBlockThreads) void insert_kernel(uint64_t* __restrict__ words, uint64_t block_mask,
                                                              KeyArgs a, uint64_t n, uint64_t n_segs,
                                                              int64_t* __restrict__ stats) {
  constexpr bool MM = K != kKeyHash;
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
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (ok[j]) {
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
    if (K != kKeyHash && !valid_at(a.validity, k)) hv = kNullHash;
    out[i] = COMBINE ? combine_hash(out[i], hv) : hv;
  }
}

// ---- k4: OR merge --------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlockThreads) void or_slices_kernel(uint64_t* __restrict__ dst,
                                                                 const uint64_t* __restrict__ srcs, uint32_t k,
                                                                 uint64_t n_words, int accumulate) {
  const uint64_t n_pairs = n_words / 2;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n_pairs; i += stride) {
    u64x2 acc = accumulate ? reinterpret_cast<const u64x2*>(dst)[i] : u64x2{0, 0};
    for (uint32_t s = 0; s < k; s++) acc |= reinterpret_cast<const u64x2*>(srcs + s * n_words)[i];
    reinterpret_cast<u64x2*>(dst)[i] = acc;
  }
  if ((n_words & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    uint64_t acc = accumulate ? dst[n_words - 1] : 0ULL;
    for (uint32_t s = 0; s < k; s++) acc |= srcs[s * n_words + n_words - 1];
    dst[n_words - 1] = acc;
  }
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

// =================================================================================================
// Host side
// =================================================================================================
struct rpt_bf {
  int device = 0;
  int log_num_blocks = 0;
  uint64_t* words = nullptr;
  uint64_t alloc_words = 0;
  int64_t* stats = nullptr;  // device {min, max} of the inserted I32/I64 keys (min/max dynamic filter)
  uint64_t sized_for_rows = 0;
  std::atomic<int> has_data{0};
  std::atomic<int> finalized{0};
  std::atomic<int> probe_strategy{RPT_PROBE_AUTO};
  std::atomic<int> insert_strategy{RPT_INSERT_AUTO};
};

namespace {

thread_local std::string t_last_error;

int fail(int status, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  t_last_error = buf;
  return status;
}

#define RPT_HIP(expr)                                                                              \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess) return fail(RPT_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

#define RPT_LAUNCHED(name)                                                                          \
  do {                                                                                              \
    hipError_t e_ = hipGetLastError();                                                              \
    if (e_ != hipSuccess) return fail(RPT_ERR_HIP, "launch of %s failed: %s", name, hipGetErrorString(e_)); \
  } while (0)

// Run device work on `device` and restore the caller's current device afterwards.
struct DeviceGuard {
  int prev = -1, target;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int d) : target(d) {
    err = hipGetDevice(&prev);
    if (err == hipSuccess && prev != d) err = hipSetDevice(d);
  }
  ~DeviceGuard() {
    if (prev >= 0 && prev != target) (void)hipSetDevice(prev);
  }
};

#define RPT_ON_DEVICE(dev)                                                                        \
  DeviceGuard guard_(dev);                                                                        \
  if (guard_.err != hipSuccess)                                                                   \
    return fail(RPT_ERR_HIP, "hipSetDevice(%d) failed: %s", (dev), hipGetErrorString(guard_.err))


// ---- kernel timing (rpt_profiling_*; mirrors rpt_profiling.hpp's counters at kernel granularity) ----
struct ProfRecord {
  const char* name;
  hipEvent_t start, end;
};
struct ProfStat {
  uint64_t launches = 0;
  double total_ms = 0.0;
};
std::atomic<int> g_prof_enabled{0};
std::mutex g_prof_mu;
std::vector<ProfRecord> g_prof_pending;
std::vector<hipEvent_t> g_prof_free;
std::vector<std::pair<std::string, ProfStat>> g_prof_stats;

hipEvent_t prof_event() {
  if (!g_prof_free.empty()) {
    hipEvent_t e = g_prof_free.back();
    g_prof_free.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// Brackets one kernel launch with events on its stream when profiling is enabled.
struct ProfScope {
  const char* name;
  hipStream_t stream;
  hipEvent_t start = nullptr;
  ProfScope(const char* n, hipStream_t s) : name(n), stream(s) {
    if (!g_prof_enabled.load(std::memory_order_relaxed)) return;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    start = prof_event();
    if (start && hipEventRecord(start, stream) != hipSuccess) start = nullptr;
  }
  void end() {
    if (!start) return;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    hipEvent_t e = prof_event();
    if (e && hipEventRecord(e, stream) == hipSuccess) {
      g_prof_pending.push_back({name, start, e});
    } else {
      g_prof_free.push_back(start);
      if (e) g_prof_free.push_back(e);
    }
    start = nullptr;
  }
};

int num_cus(int device) {
  static std::mutex mu;
  static std::vector<int> cache;
  std::lock_guard<std::mutex> lk(mu);
  if (device >= static_cast<int>(cache.size())) cache.resize(device + 1, 0);
  if (cache[device] == 0) {
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || c <= 0) c = 256;
    cache[device] = c;
  }
  return cache[device];
}

inline hipStream_t as_stream(rpt_stream_t s) { return reinterpret_cast<hipStream_t>(s); }
inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }
inline size_t align256(size_t x) { return (x + 255) & ~static_cast<size_t>(255); }

int log_blocks_for_rows(uint64_t n_rows) {
  const uint64_t bits = std::max<uint64_t>(512, n_rows > (UINT64_MAX >> 4) ? (UINT64_MAX >> 1) : n_rows * 8);
  int lg = 0;
  while (lg < 63 && (1ULL << lg) < bits) lg++;
  return lg - 6;
}

struct ProbeWorkspace {
  uint64_t* bits;
  uint32_t* seg_counts;
  uint32_t* group_sums;
  uint32_t* group_offs;
  // partitioned strategy (and level 2 of the bucketed one)
  uint32_t* recs;
  uint16_t* pos;
  uint8_t* passb;
  uint32_t* runs;     // slice-major [slice][tile]
  uint32_t* runs_tm;  // tile-major [tile][slice] (partition kernel output)
  // bucketed strategy, level 1
  uint32_t* counts_tm;     // [tile1][bucket] rows
  uint32_t* pre_bm;        // [bucket][tile1] run start inside the bucket's array
  uint32_t* pre_tm;        // [tile1][bucket] the same, tile-major
  uint32_t* totals;        // [bucket] rows
  uint64_t* bbase;         // [bucket + 1] first row of the bucket in the level-2 array
  uint32_t* bucket_tiles;  // [bucket + 1] first level-2 tile of the bucket; [nb] = level-2 tile count
  uint64_t* hashes;        // level-2 array: per bucket, its rows' hashes padded to whole tiles
  uint16_t* pos1;          // row -> position in its level-1 tile's bucket-sorted order
  uint64_t* bits2;         // level-2 result bits (level-2 array order)
};

uint32_t slice_count(int log_num_blocks) {
  return log_num_blocks <= rpt::kSliceLog ? 1u : (1u << (log_num_blocks - rpt::kSliceLog));
}

// Strategy a probe of this filter will run: explicit choice, else by filter size
// (<= 64 KiB: LDS-resident filter; <= 16 MiB: partitioned into LDS slices; larger: direct gather).
uint32_t bucket_count(int log_num_blocks) {
  return 1u << std::max(0, log_num_blocks - rpt::kSliceLog - rpt::kBucketSliceLog);
}

int strategy_supported(int strategy, int log_num_blocks) {
  constexpr int kBucketLog = rpt::kSliceLog + rpt::kBucketSliceLog;  // log2 blocks per bucket (21)
  switch (strategy) {
    case RPT_PROBE_GATHER: return 1;
    case RPT_PROBE_LDS: return log_num_blocks <= rpt::kLdsDirectMaxLog;
    case RPT_PROBE_PARTITIONED:
      return log_num_blocks >= rpt::kSliceLog && slice_count(log_num_blocks) <= static_cast<uint32_t>(rpt::kMaxSliceCount);
    case RPT_PROBE_BUCKETED:  // 2..1024 buckets of 16 MiB
      return log_num_blocks > kBucketLog && bucket_count(log_num_blocks) <= rpt::kMaxBuckets;
    default: return 0;
  }
}

// The routed strategies (partitioned, bucketed) make one pass over the whole filter (every slice is
// staged in LDS once), so they pay off only when the batch is large against the filter: n >= blocks/8
// (measured break-even against the gather: ~0.1 x blocks).
bool worth_routing(int log_num_blocks, uint64_t n) { return n >= ((1ULL << log_num_blocks) >> 3); }

// AUTO: LDS for small filters; else a routed strategy for large batches; else the gather. n = ~0 is
// "a batch of unknown, large size" (rpt_bf_probe_strategy).
int resolve_strategy(int requested, int log_num_blocks, uint64_t n) {
  if (requested != RPT_PROBE_AUTO) return requested;
  if (log_num_blocks <= rpt::kLdsDirectMaxLog) return RPT_PROBE_LDS;
  if (!worth_routing(log_num_blocks, n)) return RPT_PROBE_GATHER;
  if (strategy_supported(RPT_PROBE_PARTITIONED, log_num_blocks)) return RPT_PROBE_PARTITIONED;
  if (strategy_supported(RPT_PROBE_BUCKETED, log_num_blocks)) return RPT_PROBE_BUCKETED;
  return RPT_PROBE_GATHER;
}

// Tile-count bound of the bucketed level-2 array: every non-empty bucket pads < 1 tile.
uint64_t level2_tiles_max(uint64_t n, int log_num_blocks) {
  return ceil_div(n, rpt::kTileRows) + std::min<uint64_t>(bucket_count(log_num_blocks), n);
}

// Layout (all 256-aligned): bits | seg_counts | group_sums | group_offs, then for the partitioned
// strategy recs | pos | passb | runs | runs_tm (whole 16 Ki-row tiles), and for the bucketed one the
// same level-2 arrays over level2_tiles_max tiles of 128 slices plus the level-1 arrays.
size_t workspace_layout(uint64_t n, int log_num_blocks, int strategy, void* base, ProbeWorkspace* ws) {
  const uint64_t n_segs = ceil_div(n, rpt::kSegRows);
  const uint64_t n_groups = ceil_div(n_segs, rpt::kGroupSegs);
  const uint64_t T = rpt::kTileRows;
  constexpr int kParts = 19;
  size_t sz[kParts] = {align256(n_segs * rpt::kWordsPerSeg * 8), align256(n_groups * rpt::kGroupSegs * 4),
                       align256(n_groups * 4), align256(n_groups * 4)};
  const bool part = strategy == RPT_PROBE_PARTITIONED, buck = strategy == RPT_PROBE_BUCKETED;
  if (part || buck) {
    const uint64_t tiles = part ? ceil_div(n, T) : level2_tiles_max(n, log_num_blocks);
    const uint32_t slices = part ? slice_count(log_num_blocks) : rpt::kBucketSlices;
    const uint64_t cap = rpt::tile_cap_for(slices);
    sz[4] = align256(tiles * cap * 4);
    sz[5] = align256(tiles * T * 2);
    sz[6] = align256(tiles * cap / 8);
    sz[7] = align256(static_cast<uint64_t>(slices) * tiles * 4);
    sz[8] = sz[7];
  }
  if (buck) {
    const uint64_t t1 = ceil_div(n, T), t2 = level2_tiles_max(n, log_num_blocks);
    const uint64_t nb = bucket_count(log_num_blocks);
    sz[9] = sz[10] = sz[11] = align256(t1 * nb * 4);
    sz[12] = align256(nb * 4);
    sz[13] = align256((nb + 1) * 8);
    sz[14] = align256((nb + 1) * 4);
    sz[15] = align256(t2 * T * 8);
    sz[16] = align256(t1 * T * 2);
    sz[17] = align256(t2 * T / 8);
  }
  size_t off[kParts], total = 0;
  for (int i = 0; i < kParts; i++) {
    off[i] = total;
    total += sz[i];
  }
  if (ws) {
    char* p = static_cast<char*>(base);
    auto at = [&](int i) -> void* { return sz[i] ? p + off[i] : nullptr; };
    ws->bits = static_cast<uint64_t*>(at(0));
    ws->seg_counts = static_cast<uint32_t*>(at(1));
    ws->group_sums = static_cast<uint32_t*>(at(2));
    ws->group_offs = static_cast<uint32_t*>(at(3));
    ws->recs = static_cast<uint32_t*>(at(4));
    ws->pos = static_cast<uint16_t*>(at(5));
    ws->passb = static_cast<uint8_t*>(at(6));
    ws->runs = static_cast<uint32_t*>(at(7));
    ws->runs_tm = static_cast<uint32_t*>(at(8));
    ws->counts_tm = static_cast<uint32_t*>(at(9));
    ws->pre_bm = static_cast<uint32_t*>(at(10));
    ws->pre_tm = static_cast<uint32_t*>(at(11));
    ws->totals = static_cast<uint32_t*>(at(12));
    ws->bbase = static_cast<uint64_t*>(at(13));
    ws->bucket_tiles = static_cast<uint32_t*>(at(14));
    ws->hashes = static_cast<uint64_t*>(at(15));
    ws->pos1 = static_cast<uint16_t*>(at(16));
    ws->bits2 = static_cast<uint64_t*>(at(17));
  }
  return total;
}

// Build workspace: records | runs (slice-major) | runs (tile-major) (partitioned, or level 2 of the
// bucketed insert), then the bucketed level-1 arrays.
struct InsertWorkspace {
  uint32_t* recs;
  uint32_t* runs;
  uint32_t* runs_tm;
  uint32_t* counts_tm;
  uint32_t* pre_bm;
  uint32_t* pre_tm;
  uint32_t* totals;
  uint64_t* bbase;
  uint32_t* bucket_tiles;
  uint64_t* hashes;
};

size_t insert_workspace_layout(uint64_t n, int log_num_blocks, int strategy, void* base, InsertWorkspace* ws) {
  const bool buck = strategy == RPT_INSERT_BUCKETED;
  if (strategy != RPT_INSERT_PARTITIONED && !buck) return 0;
  const uint64_t T = rpt::kTileRows;
  const uint64_t tiles = buck ? level2_tiles_max(n, log_num_blocks) : ceil_div(n, T);
  const uint32_t slices = buck ? rpt::kBucketSlices : slice_count(log_num_blocks);
  constexpr int kParts = 10;
  size_t sz[kParts] = {align256(tiles * rpt::tile_cap_for(slices) * 4), align256(static_cast<uint64_t>(slices) * tiles * 4),
                       align256(static_cast<uint64_t>(slices) * tiles * 4)};
  if (buck) {
    const uint64_t t1 = ceil_div(n, T), nb = bucket_count(log_num_blocks);
    sz[3] = sz[4] = sz[5] = align256(t1 * nb * 4);
    sz[6] = align256(nb * 4);
    sz[7] = align256((nb + 1) * 8);
    sz[8] = align256((nb + 1) * 4);
    sz[9] = align256(tiles * T * 8);
  }
  size_t off[kParts], total = 0;
  for (int i = 0; i < kParts; i++) {
    off[i] = total;
    total += sz[i];
  }
  if (ws) {
    char* p = static_cast<char*>(base);
    auto at = [&](int i) -> void* { return sz[i] ? p + off[i] : nullptr; };
    ws->recs = static_cast<uint32_t*>(at(0));
    ws->runs = static_cast<uint32_t*>(at(1));
    ws->runs_tm = static_cast<uint32_t*>(at(2));
    ws->counts_tm = static_cast<uint32_t*>(at(3));
    ws->pre_bm = static_cast<uint32_t*>(at(4));
    ws->pre_tm = static_cast<uint32_t*>(at(5));
    ws->totals = static_cast<uint32_t*>(at(6));
    ws->bbase = static_cast<uint64_t*>(at(7));
    ws->bucket_tiles = static_cast<uint32_t*>(at(8));
    ws->hashes = static_cast<uint64_t*>(at(9));
  }
  return total;
}

constexpr uint64_t kPartitionedInsertMinRows = 1ULL << 20;

int resolve_insert_strategy(int requested, int log_num_blocks, uint64_t n) {
  if (requested != RPT_INSERT_AUTO) return requested;
  if (n < kPartitionedInsertMinRows) return RPT_INSERT_ATOMIC;
  if (strategy_supported(RPT_PROBE_PARTITIONED, log_num_blocks)) return RPT_INSERT_PARTITIONED;
  if (strategy_supported(RPT_PROBE_BUCKETED, log_num_blocks) && worth_routing(log_num_blocks, n))
    return RPT_INSERT_BUCKETED;
  return RPT_INSERT_ATOMIC;
}

int check_col(const rpt_key_column* col) {
  if (!col) return fail(RPT_ERR_INVALID_ARGUMENT, "null key column");
  if (col->key_type < RPT_KEY_I64 || col->key_type > RPT_KEY_HASH)
    return fail(RPT_ERR_INVALID_ARGUMENT, "bad key_type %d", col->key_type);
  if (!col->keys) return fail(RPT_ERR_INVALID_ARGUMENT, "null keys pointer");
  return RPT_OK;
}

bool dense_ok(const rpt_key_column* col, const uint32_t* row_sel) {
  return row_sel == nullptr && col->key_sel == nullptr && (reinterpret_cast<uintptr_t>(col->keys) & 15) == 0;
}

unsigned persistent_grid(int device, uint64_t n_segs) {
  const uint64_t want = ceil_div(n_segs, rpt::kWavesPerBlock);
  const uint64_t cap = static_cast<uint64_t>(num_cus(device)) * rpt::kBlocksPerCU;
  return static_cast<unsigned>(std::max<uint64_t>(1, std::min(want, cap)));
}

template <int K, bool D>
void launch_probe_bits_t(unsigned grid, hipStream_t s, const rpt_bf* bf, const rpt::KeyArgs& a, uint64_t n,
                         uint64_t n_segs, uint64_t* bits, uint32_t* counts) {
  hipLaunchKernelGGL((rpt::probe_bits_kernel<K, D, false>), dim3(grid), dim3(rpt::kBlockThreads), 0, s, bf->words,
                     (1ULL << bf->log_num_blocks) - 1, a, n, n_segs, bits, counts);
}

// Whole filter in LDS (dynamic LDS = filter bytes); as many workgroups per CU as LDS allows.
template <int K, bool D>
void launch_probe_bits_lds_t(unsigned grid, hipStream_t s, const rpt_bf* bf, const rpt::KeyArgs& a, uint64_t n,
                             uint64_t n_segs, uint64_t* bits, uint32_t* counts) {
  const size_t lds = 8ULL << bf->log_num_blocks;
  hipLaunchKernelGGL((rpt::probe_bits_kernel<K, D, true>), dim3(grid), dim3(rpt::kBlockThreads), lds, s, bf->words,
                     (1ULL << bf->log_num_blocks) - 1, a, n, n_segs, bits, counts);
}

// Let `fn` use all of the CU's 160 KiB of LDS: dynamic allowance = 160 KiB - its static LDS.
void allow_dynamic_lds(const void* fn) {
  hipFuncAttributes at{};
  size_t stat = 0;
  if (hipFuncGetAttributes(&at, fn) == hipSuccess) stat = at.sharedSizeBytes;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>((160u << 10) - stat));
  (void)hipGetLastError();
}

template <int K, bool D, bool MM>
void launch_partition_mm(unsigned grid, hipStream_t s, const rpt::KeyArgs& a, uint64_t n, uint32_t slice_mask,
                         uint64_t n_tiles, uint32_t* recs, uint16_t* pos, uint32_t* runs, int64_t* stats,
                         const uint32_t* dev_n_tiles = nullptr) {
  const uint32_t slices = slice_mask + 1;
  const size_t lds = rpt::tile_cap_for(slices) * 4 + 2ULL * slices * 4;
  static std::once_flag once;  // per instantiation; > 64 KiB of dynamic LDS must be opted into
  std::call_once(once, [] { allow_dynamic_lds(reinterpret_cast<const void*>(&rpt::partition_kernel<K, D, MM>)); });
  hipLaunchKernelGGL((rpt::partition_kernel<K, D, MM>), dim3(grid), dim3(rpt::kTileThreads), lds, s, a, n, slice_mask,
                     n_tiles, recs, pos, runs, stats, dev_n_tiles);
}

// stats == nullptr: probe (no min/max); otherwise the build's key min/max is folded into stats.
template <int K, bool D>
void launch_partition_t(unsigned grid, hipStream_t s, const rpt::KeyArgs& a, uint64_t n, uint32_t slice_mask,
                        uint64_t n_tiles, uint32_t* recs, uint16_t* pos, uint32_t* runs, int64_t* stats,
                        const uint32_t* dev_n_tiles) {
  if (K != rpt::kKeyHash && stats != nullptr)
    launch_partition_mm<K, D, true>(grid, s, a, n, slice_mask, n_tiles, recs, pos, runs, stats, dev_n_tiles);
  else
    launch_partition_mm<K, D, false>(grid, s, a, n, slice_mask, n_tiles, recs, pos, runs, nullptr, dev_n_tiles);
}

template <int K, bool D>
void launch_insert_t(unsigned grid, hipStream_t s, rpt_bf* bf, const rpt::KeyArgs& a, uint64_t n, uint64_t n_segs) {
  hipLaunchKernelGGL((rpt::insert_kernel<K, D>), dim3(grid), dim3(rpt::kBlockThreads), 0, s, bf->words,
                     (1ULL << bf->log_num_blocks) - 1, a, n, n_segs, bf->stats);
}

template <int K, bool D>
void launch_bucket_count_t(unsigned grid, hipStream_t s, const rpt::KeyArgs& a, uint64_t n, uint32_t bucket_mask,
                           uint32_t* counts_tm, int64_t* stats) {
  if (K != rpt::kKeyHash && stats != nullptr)
    hipLaunchKernelGGL((rpt::bucket_count_kernel<K, D, true>), dim3(grid), dim3(rpt::kTileThreads), 0, s, a, n,
                       bucket_mask, counts_tm, stats);
  else
    hipLaunchKernelGGL((rpt::bucket_count_kernel<K, D, false>), dim3(grid), dim3(rpt::kTileThreads), 0, s, a, n,
                       bucket_mask, counts_tm, static_cast<int64_t*>(nullptr));
}

template <int K, bool D>
void launch_bucket_scatter_t(unsigned grid, hipStream_t s, const rpt::KeyArgs& a, uint64_t n, uint32_t bucket_mask,
                             const uint32_t* counts_tm, const uint32_t* pre_tm, const uint64_t* bbase, uint64_t* hashes,
                             uint16_t* pos1) {
  const size_t lds = rpt::kTileRows * 8;
  static std::once_flag once;  // > 64 KiB of dynamic LDS must be opted into (160 KiB minus the static part)
  std::call_once(once, [] { allow_dynamic_lds(reinterpret_cast<const void*>(&rpt::bucket_scatter_kernel<K, D>)); });
  hipLaunchKernelGGL((rpt::bucket_scatter_kernel<K, D>), dim3(grid), dim3(rpt::kTileThreads), lds, s, a, n, bucket_mask,
                     counts_tm, pre_tm, bbase, hashes, pos1);
}

#define RPT_DISPATCH_KD(fn, kt, dense, ...)                  \
  do {                                                       \
    switch (kt) {                                            \
      case RPT_KEY_I64:                                      \
        if (dense) fn<rpt::kKeyI64, true>(__VA_ARGS__);      \
        else fn<rpt::kKeyI64, false>(__VA_ARGS__);           \
        break;                                               \
      case RPT_KEY_I32:                                      \
        if (dense) fn<rpt::kKeyI32, true>(__VA_ARGS__);      \
        else fn<rpt::kKeyI32, false>(__VA_ARGS__);           \
        break;                                               \
      default:                                               \
        if (dense) fn<rpt::kKeyHash, true>(__VA_ARGS__);     \
        else fn<rpt::kKeyHash, false>(__VA_ARGS__);          \
        break;                                               \
    }                                                        \
  } while (0)

// [rows][cols] u32 matrix -> [cols][rows] (the run-table transpose kernel).
int transpose_u32(hipStream_t s, const uint32_t* in, uint64_t rows, uint64_t cols, uint32_t* out) {
  if (ceil_div(cols, 64) > 65535) return fail(RPT_ERR_INVALID_ARGUMENT, "transpose of %llu columns", (unsigned long long)cols);
  ProfScope prof_t("runs_transpose_kernel", s);
  hipLaunchKernelGGL(rpt::runs_transpose_kernel, dim3(static_cast<unsigned>(ceil_div(rows, 64)), static_cast<unsigned>(ceil_div(cols, 64))),
                     dim3(rpt::kBlockThreads), 0, s, in, static_cast<uint32_t>(cols), rows, out);
  prof_t.end();
  RPT_LAUNCHED("runs_transpose_kernel");
  return RPT_OK;
}

// Level 1 of the bucketed strategies: rows per (tile, bucket) [+ the build's min/max], the buckets'
// prefix tables and bases, every row's hash copied into its bucket's array (+ its position in the
// tile's bucket-sorted order when pos1 != nullptr), each array padded to whole tiles.
struct BucketLevel1 {
  uint32_t *counts_tm, *pre_bm, *pre_tm, *totals, *bucket_tiles;
  uint64_t *bbase, *hashes;
  uint16_t* pos1;
};
int run_bucket_level1(hipStream_t s, int key_type, const rpt::KeyArgs& a, bool dense, uint64_t n, int L,
                      const BucketLevel1& w, int64_t* stats) {
  const uint32_t nb = bucket_count(L);
  const uint64_t t1 = ceil_div(n, rpt::kTileRows);
  {
    ProfScope prof_c("bucket_count_kernel", s);
    RPT_DISPATCH_KD(launch_bucket_count_t, key_type, dense, static_cast<unsigned>(t1), s, a, n, nb - 1, w.counts_tm, stats);
    prof_c.end();
    RPT_LAUNCHED("bucket_count_kernel");
  }
  int st = transpose_u32(s, w.counts_tm, t1, nb, w.pre_bm);
  if (st != RPT_OK) return st;
  {
    ProfScope prof_s("bucket_scan_kernel", s);
    hipLaunchKernelGGL(rpt::bucket_scan_kernel, dim3(nb), dim3(1024), 0, s, w.pre_bm, t1, w.totals);
    hipLaunchKernelGGL(rpt::bucket_base_kernel, dim3(1), dim3(1024), 0, s, w.totals, nb, w.bbase, w.bucket_tiles);
    prof_s.end();
    RPT_LAUNCHED("bucket_scan_kernel");
  }
  st = transpose_u32(s, w.pre_bm, nb, t1, w.pre_tm);
  if (st != RPT_OK) return st;
  {
    ProfScope prof_x("bucket_scatter_kernel", s);
    RPT_DISPATCH_KD(launch_bucket_scatter_t, key_type, dense, static_cast<unsigned>(t1), s, a, n, nb - 1, w.counts_tm,
                    w.pre_tm, w.bbase, w.hashes, w.pos1);
    hipLaunchKernelGGL(rpt::bucket_pad_kernel, dim3(nb), dim3(rpt::kBlockThreads), 0, s, w.totals, w.bbase, w.hashes);
    prof_x.end();
    RPT_LAUNCHED("bucket_scatter_kernel");
  }
  return RPT_OK;
}

int alloc_words(rpt_bf* bf, int log_nb) {
  const uint64_t nw = 1ULL << log_nb;
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, nw * 8);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return fail(RPT_ERR_OUT_OF_MEMORY, "hipMalloc(%llu bytes) failed: %s", static_cast<unsigned long long>(nw * 8),
                hipGetErrorString(e));
  }
  e = hipMemset(p, 0, nw * 8);
  if (e != hipSuccess) {
    (void)hipFree(p);
    return fail(RPT_ERR_HIP, "hipMemset failed: %s", hipGetErrorString(e));
  }
  bf->words = static_cast<uint64_t*>(p);
  bf->alloc_words = nw;
  bf->log_num_blocks = log_nb;
  return RPT_OK;
}

const int64_t kStatsInit[2] = {INT64_MAX, INT64_MIN};

int alloc_stats(rpt_bf* bf) {
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, sizeof kStatsInit);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return fail(RPT_ERR_OUT_OF_MEMORY, "hipMalloc(stats) failed: %s", hipGetErrorString(e));
  }
  bf->stats = static_cast<int64_t*>(p);
  e = hipMemcpy(bf->stats, kStatsInit, sizeof kStatsInit, hipMemcpyHostToDevice);
  if (e != hipSuccess) return fail(RPT_ERR_HIP, "stats init failed: %s", hipGetErrorString(e));
  return RPT_OK;
}

// {min, max} reset on the stream (after the caller's earlier work on it)
__global__ void stats_reset_kernel(int64_t* stats) {
  stats[0] = INT64_MAX;
  stats[1] = INT64_MIN;
}
__global__ void stats_merge_kernel(int64_t* dst, const int64_t* src) {
  if (src[0] < dst[0]) dst[0] = src[0];
  if (src[1] > dst[1]) dst[1] = src[1];
}

}  // namespace

namespace {
template <bool COMBINE>
int launch_hash(const rpt_key_column* col, uint64_t n, uint64_t* out_hashes, rpt_stream_t stream) {
  if (!out_hashes) return fail(RPT_ERR_INVALID_ARGUMENT, "null out");
  if (n == 0) return RPT_OK;
  int st = check_col(col);
  if (st != RPT_OK) return st;
  const unsigned grid = static_cast<unsigned>(std::min<uint64_t>(ceil_div(n, rpt::kBlockThreads), 4096));
  const rpt::KeyArgs a{col->keys, col->key_sel, col->validity, nullptr};
  hipStream_t s = as_stream(stream);
  ProfScope prof_("hash_kernel", s);
  switch (col->key_type) {
    case RPT_KEY_I64: hipLaunchKernelGGL((rpt::hash_kernel<rpt::kKeyI64, COMBINE>), dim3(grid), dim3(rpt::kBlockThreads), 0, s, a, n, out_hashes); break;
    case RPT_KEY_I32: hipLaunchKernelGGL((rpt::hash_kernel<rpt::kKeyI32, COMBINE>), dim3(grid), dim3(rpt::kBlockThreads), 0, s, a, n, out_hashes); break;
    default: hipLaunchKernelGGL((rpt::hash_kernel<rpt::kKeyHash, COMBINE>), dim3(grid), dim3(rpt::kBlockThreads), 0, s, a, n, out_hashes); break;
  }
  prof_.end();
  RPT_LAUNCHED("hash_kernel");
  return RPT_OK;
}
}  // namespace

extern "C" {

int rpt_abi_version(void) { return RPT_GPU_ABI_VERSION; }

const char* rpt_status_string(int status) {
  switch (status) {
    case RPT_OK: return "ok";
    case RPT_ERR_INVALID_ARGUMENT: return "invalid argument";
    case RPT_ERR_HIP: return "HIP runtime error";
    case RPT_ERR_OUT_OF_MEMORY: return "out of device memory";
    case RPT_ERR_WORKSPACE: return "workspace too small";
    case RPT_ERR_SHAPE_MISMATCH: return "filter shape mismatch";
    default: return "unknown status";
  }
}

const char* rpt_last_error(void) { return t_last_error.c_str(); }

int rpt_bf_log_num_blocks_for_rows(uint64_t n_rows) { return log_blocks_for_rows(n_rows); }

int rpt_bf_needs_resize(uint64_t sized_for_rows, uint64_t actual_rows) {
  if (actual_rows == 0) return 0;
  const uint64_t min_bits = std::max<uint64_t>(512, sized_for_rows * 12);
  uint64_t alloc = 1;
  while (alloc < min_bits) alloc <<= 1;
  return actual_rows * 8 > alloc ? 1 : 0;
}

size_t rpt_probe_workspace_bytes(uint64_t n_rows, int log_num_blocks) {
  // enough for any strategy the filter may run
  size_t m = 0;
  for (int st : {RPT_PROBE_GATHER, RPT_PROBE_LDS, RPT_PROBE_PARTITIONED, RPT_PROBE_BUCKETED})
    if (strategy_supported(st, log_num_blocks)) m = std::max(m, workspace_layout(n_rows, log_num_blocks, st, nullptr, nullptr));
  return m;
}

int rpt_bf_probe_strategy_for(const rpt_bf* bf, uint64_t n_rows) {
  if (!bf) return -fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  return resolve_strategy(bf->probe_strategy.load(), bf->log_num_blocks, n_rows);
}

size_t rpt_bf_probe_workspace_bytes(const rpt_bf* bf, uint64_t n_rows) {
  if (!bf) return 0;
  const int st = resolve_strategy(bf->probe_strategy.load(), bf->log_num_blocks, n_rows);
  return workspace_layout(n_rows, bf->log_num_blocks, st, nullptr, nullptr);
}

int rpt_probe_strategy_supported(int strategy, int log_num_blocks) {
  return strategy == RPT_PROBE_AUTO ? 1 : strategy_supported(strategy, log_num_blocks);
}

int rpt_bf_set_probe_strategy(rpt_bf* bf, int strategy) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  if (strategy < RPT_PROBE_AUTO || strategy > RPT_PROBE_BUCKETED)
    return fail(RPT_ERR_INVALID_ARGUMENT, "unknown probe strategy %d", strategy);
  bf->probe_strategy.store(strategy);
  return RPT_OK;
}

int rpt_bf_probe_strategy(const rpt_bf* bf) {
  if (!bf) return -fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  return resolve_strategy(bf->probe_strategy.load(), bf->log_num_blocks, ~0ULL);
}

int rpt_bf_create_log_blocks(int device, int log_num_blocks, rpt_bf** out) {
  if (!out) return fail(RPT_ERR_INVALID_ARGUMENT, "null out");
  *out = nullptr;
  if (log_num_blocks < 0 || log_num_blocks > 40) return fail(RPT_ERR_INVALID_ARGUMENT, "log_num_blocks %d", log_num_blocks);
  RPT_ON_DEVICE(device);
  rpt_bf* bf = new rpt_bf();
  bf->device = device;
  int st = alloc_words(bf, log_num_blocks);
  if (st == RPT_OK) st = alloc_stats(bf);
  if (st != RPT_OK) {
    if (bf->words) (void)hipFree(bf->words);
    delete bf;
    return st;
  }
  *out = bf;
  return RPT_OK;
}

int rpt_bf_create(int device, uint64_t est_num_rows, rpt_bf** out) {
  int st = rpt_bf_create_log_blocks(device, log_blocks_for_rows(est_num_rows), out);
  if (st == RPT_OK) (*out)->sized_for_rows = est_num_rows;
  return st;
}

int rpt_bf_destroy(rpt_bf* bf) {
  if (!bf) return RPT_OK;
  {
    DeviceGuard g(bf->device);
    if (bf->words) (void)hipFree(bf->words);
    if (bf->stats) (void)hipFree(bf->stats);
  }
  delete bf;
  return RPT_OK;
}

int rpt_bf_get_info(const rpt_bf* bf, rpt_bf_info* out) {
  if (!bf || !out) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  out->device = bf->device;
  out->log_num_blocks = bf->log_num_blocks;
  out->num_blocks = 1ULL << bf->log_num_blocks;
  out->sized_for_rows = bf->sized_for_rows;
  out->has_data = bf->has_data.load();
  out->finalized = bf->finalized.load();
  out->words = bf->words;
  return RPT_OK;
}

int rpt_bf_reinitialize(rpt_bf* bf, uint64_t actual_rows) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  RPT_ON_DEVICE(bf->device);
  RPT_HIP(hipDeviceSynchronize());
  if (bf->words) RPT_HIP(hipFree(bf->words));
  bf->words = nullptr;
  int st = alloc_words(bf, log_blocks_for_rows(actual_rows));
  if (st != RPT_OK) return st;
  bf->sized_for_rows = actual_rows;
  bf->has_data.store(0);
  RPT_HIP(hipMemcpy(bf->stats, kStatsInit, sizeof kStatsInit, hipMemcpyHostToDevice));
  return RPT_OK;
}

int rpt_bf_set_finalized(rpt_bf* bf, int value) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  bf->finalized.store(value ? 1 : 0);
  return RPT_OK;
}

int rpt_bf_set_has_data(rpt_bf* bf, int value) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  bf->has_data.store(value ? 1 : 0);
  return RPT_OK;
}

int rpt_bf_clear(rpt_bf* bf, rpt_stream_t stream) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  RPT_ON_DEVICE(bf->device);
  RPT_HIP(hipMemsetAsync(bf->words, 0, (1ULL << bf->log_num_blocks) * 8, as_stream(stream)));
  hipLaunchKernelGGL(stats_reset_kernel, dim3(1), dim3(1), 0, as_stream(stream), bf->stats);
  RPT_LAUNCHED("stats_reset_kernel");
  bf->has_data.store(0);
  return RPT_OK;
}

int rpt_bf_get_minmax(const rpt_bf* bf, int64_t* out_min, int64_t* out_max, int* out_has_value, rpt_stream_t stream) {
  if (!bf || !out_min || !out_max || !out_has_value) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  RPT_ON_DEVICE(bf->device);
  int64_t v[2];
  RPT_HIP(hipMemcpyAsync(v, bf->stats, sizeof v, hipMemcpyDeviceToHost, as_stream(stream)));
  RPT_HIP(hipStreamSynchronize(as_stream(stream)));
  *out_has_value = v[0] <= v[1] ? 1 : 0;
  *out_min = *out_has_value ? v[0] : 0;
  *out_max = *out_has_value ? v[1] : 0;
  return RPT_OK;
}

int rpt_bf_set_minmax(rpt_bf* bf, int64_t min_value, int64_t max_value, int has_value, rpt_stream_t stream) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  if (has_value && min_value > max_value) return fail(RPT_ERR_INVALID_ARGUMENT, "min > max");
  RPT_ON_DEVICE(bf->device);
  static thread_local int64_t v[2];  // pageable source: hipMemcpyAsync copies it before returning
  v[0] = has_value ? min_value : INT64_MAX;
  v[1] = has_value ? max_value : INT64_MIN;
  RPT_HIP(hipMemcpyAsync(bf->stats, v, sizeof v, hipMemcpyHostToDevice, as_stream(stream)));
  RPT_HIP(hipStreamSynchronize(as_stream(stream)));
  return RPT_OK;
}

int rpt_bf_insert(rpt_bf* bf, const rpt_key_column* col, uint64_t n, rpt_stream_t stream) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  if (n == 0) return RPT_OK;  // bloom_filter.cpp:72-74
  int st = check_col(col);
  if (st != RPT_OK) return st;
  RPT_ON_DEVICE(bf->device);
  bf->has_data.store(1);  // bloom_filter.cpp:75
  const uint64_t n_segs = ceil_div(n, rpt::kSegRows);
  const unsigned grid = persistent_grid(bf->device, n_segs);
  const rpt::KeyArgs a{col->keys, col->key_sel, col->validity, nullptr};
  ProfScope prof1_("insert_kernel", as_stream(stream));
  RPT_DISPATCH_KD(launch_insert_t, col->key_type, dense_ok(col, nullptr), grid, as_stream(stream), bf, a, n, n_segs);
  prof1_.end();
  RPT_LAUNCHED("insert_kernel");
  return RPT_OK;
}

size_t rpt_insert_workspace_bytes(uint64_t n_rows, int log_num_blocks) {
  size_t m = 0;
  if (strategy_supported(RPT_PROBE_PARTITIONED, log_num_blocks))
    m = std::max(m, insert_workspace_layout(n_rows, log_num_blocks, RPT_INSERT_PARTITIONED, nullptr, nullptr));
  if (strategy_supported(RPT_PROBE_BUCKETED, log_num_blocks))
    m = std::max(m, insert_workspace_layout(n_rows, log_num_blocks, RPT_INSERT_BUCKETED, nullptr, nullptr));
  return m;
}

int rpt_bf_insert_strategy_for(const rpt_bf* bf, uint64_t n_rows) {
  if (!bf) return -fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  return resolve_insert_strategy(bf->insert_strategy.load(), bf->log_num_blocks, n_rows);
}

size_t rpt_bf_insert_workspace_bytes(const rpt_bf* bf, uint64_t n_rows) {
  if (!bf) return 0;
  const int st = resolve_insert_strategy(bf->insert_strategy.load(), bf->log_num_blocks, n_rows);
  return insert_workspace_layout(n_rows, bf->log_num_blocks, st, nullptr, nullptr);
}

int rpt_bf_set_insert_strategy(rpt_bf* bf, int strategy) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  if (strategy < RPT_INSERT_AUTO || strategy > RPT_INSERT_BUCKETED)
    return fail(RPT_ERR_INVALID_ARGUMENT, "unknown insert strategy %d", strategy);
  bf->insert_strategy.store(strategy);
  return RPT_OK;
}

int rpt_bf_insert_ws(rpt_bf* bf, const rpt_key_column* col, uint64_t n, void* workspace, size_t workspace_bytes,
                     rpt_stream_t stream) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  if (n == 0) return RPT_OK;  // bloom_filter.cpp:72-74
  const int L = bf->log_num_blocks;
  const int strategy = resolve_insert_strategy(bf->insert_strategy.load(), L, n);
  if (strategy == RPT_INSERT_ATOMIC) return rpt_bf_insert(bf, col, n, stream);
  const bool buck = strategy == RPT_INSERT_BUCKETED;
  if (!strategy_supported(buck ? RPT_PROBE_BUCKETED : RPT_PROBE_PARTITIONED, L))
    return fail(RPT_ERR_INVALID_ARGUMENT, "%s insert unsupported for a 2^%d-block filter",
                buck ? "bucketed" : "partitioned", L);
  int st = check_col(col);
  if (st != RPT_OK) return st;
  const size_t need = insert_workspace_layout(n, L, strategy, nullptr, nullptr);
  if (!workspace || workspace_bytes < need)
    return fail(RPT_ERR_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes, need);
  RPT_ON_DEVICE(bf->device);
  bf->has_data.store(1);  // bloom_filter.cpp:75
  InsertWorkspace ws;
  insert_workspace_layout(n, L, strategy, workspace, &ws);
  hipStream_t s = as_stream(stream);
  const int cus = num_cus(bf->device);
  const rpt::KeyArgs a{col->keys, col->key_sel, col->validity, nullptr};
  const bool dense = dense_ok(col, nullptr);
  // the partition input: the key column itself, or (bucketed) the level-2 hash array
  uint32_t tile_slices = slice_count(L);
  uint64_t n_tiles = ceil_div(n, rpt::kTileRows), n_part = n;
  rpt::KeyArgs pa = a;
  int p_type = col->key_type;
  bool p_dense = dense;
  int64_t* p_stats = bf->stats;
  const uint32_t* bucket_tiles = nullptr;
  const uint32_t* dev_n_tiles = nullptr;
  uint32_t grid_slices = tile_slices;
  if (buck) {
    const BucketLevel1 l1{ws.counts_tm, ws.pre_bm, ws.pre_tm, ws.totals, ws.bucket_tiles, ws.bbase, ws.hashes, nullptr};
    st = run_bucket_level1(s, col->key_type, a, dense, n, L, l1, bf->stats);
    if (st != RPT_OK) return st;
    tile_slices = rpt::kBucketSlices;
    n_tiles = level2_tiles_max(n, L);
    n_part = n_tiles * rpt::kTileRows;
    pa = rpt::KeyArgs{ws.hashes, nullptr, nullptr, nullptr};
    p_type = RPT_KEY_HASH;
    p_dense = true;
    p_stats = nullptr;  // min/max came from the key read of level 1
    bucket_tiles = ws.bucket_tiles;
    dev_n_tiles = ws.bucket_tiles + bucket_count(L);
    grid_slices = bucket_count(L) * rpt::kBucketSlices;
  }
  ProfScope prof_p("partition_kernel", s);
  RPT_DISPATCH_KD(launch_partition_t, p_type, p_dense, static_cast<unsigned>(n_tiles), s, pa, n_part, tile_slices - 1,
                  n_tiles, ws.recs, static_cast<uint16_t*>(nullptr), ws.runs_tm, p_stats, dev_n_tiles);
  prof_p.end();
  RPT_LAUNCHED("partition_kernel");
  st = transpose_u32(s, ws.runs_tm, n_tiles, tile_slices, ws.runs);
  if (st != RPT_OK) return st;
  const uint32_t splits = static_cast<uint32_t>(
      std::max<uint64_t>(1, std::min<uint64_t>(n_tiles, static_cast<uint64_t>(cus) / grid_slices)));
  ProfScope prof_i("slice_insert_kernel", s);
  hipLaunchKernelGGL(rpt::slice_insert_kernel, dim3(grid_slices * splits), dim3(rpt::kSliceThreads), 0, s, bf->words, splits,
                     n_tiles, ws.recs, ws.runs, tile_slices, bucket_tiles);
  prof_i.end();
  RPT_LAUNCHED("slice_insert_kernel");
  return RPT_OK;
}

int rpt_bf_find_bits(const rpt_bf* bf, const rpt_key_column* col, uint64_t n, uint64_t* out_bits,
                     rpt_stream_t stream) {
  if (!bf || !out_bits) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  if (n == 0) return RPT_OK;
  int st = check_col(col);
  if (st != RPT_OK) return st;
  RPT_ON_DEVICE(bf->device);
  const uint64_t n_segs = ceil_div(n, rpt::kSegRows);
  const unsigned grid = persistent_grid(bf->device, n_segs);
  const rpt::KeyArgs a{col->keys, col->key_sel, col->validity, nullptr};
  ProfScope prof2_("probe_bits_kernel", as_stream(stream));
  RPT_DISPATCH_KD(launch_probe_bits_t, col->key_type, dense_ok(col, nullptr), grid, as_stream(stream), bf, a, n,
                  n_segs, out_bits, static_cast<uint32_t*>(nullptr));
  prof2_.end();
  RPT_LAUNCHED("probe_bits_kernel");
  return RPT_OK;
}

int rpt_bf_probe_phase1(const rpt_bf* bf, const rpt_key_column* col, const uint32_t* row_sel, uint64_t n,
                        void* workspace, size_t workspace_bytes, rpt_stream_t stream) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  if (n >= (1ULL << 32)) return fail(RPT_ERR_INVALID_ARGUMENT, "n=%llu rows exceeds uint32 sel_t", (unsigned long long)n);
  if (n == 0) return RPT_OK;
  int st = check_col(col);
  if (st != RPT_OK) return st;
  const int L = bf->log_num_blocks;
  const int strategy = resolve_strategy(bf->probe_strategy.load(), L, n);
  if (!strategy_supported(strategy, L))
    return fail(RPT_ERR_INVALID_ARGUMENT, "probe strategy %d unsupported for a 2^%d-block filter", strategy, L);
  const size_t need = workspace_layout(n, L, strategy, nullptr, nullptr);
  if (!workspace || workspace_bytes < need)
    return fail(RPT_ERR_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes, need);
  RPT_ON_DEVICE(bf->device);
  ProbeWorkspace ws;
  workspace_layout(n, L, strategy, workspace, &ws);
  hipStream_t s = as_stream(stream);
  const uint64_t n_segs = ceil_div(n, rpt::kSegRows);
  const rpt::KeyArgs a{col->keys, col->key_sel, col->validity, row_sel};
  const bool dense = dense_ok(col, row_sel);
  if (strategy == RPT_PROBE_GATHER) {
    const unsigned grid = persistent_grid(bf->device, n_segs);
    ProfScope prof3_("probe_bits_kernel", s);
    RPT_DISPATCH_KD(launch_probe_bits_t, col->key_type, dense, grid, s, bf, a, n, n_segs, ws.bits, ws.seg_counts);
    prof3_.end();
    RPT_LAUNCHED("probe_bits_kernel");
  } else if (strategy == RPT_PROBE_LDS) {
    const uint64_t lds = (8ULL << L) + 8ULL * rpt::kNumMasks;
    const uint64_t per_cu = std::max<uint64_t>(1, std::min<uint64_t>(rpt::kBlocksPerCU, (160ULL << 10) / lds));
    const unsigned grid = static_cast<unsigned>(
        std::max<uint64_t>(1, std::min(ceil_div(n_segs, rpt::kWavesPerBlock), num_cus(bf->device) * per_cu)));
    ProfScope prof4_("probe_bits_kernel<lds>", s);
    RPT_DISPATCH_KD(launch_probe_bits_lds_t, col->key_type, dense, grid, s, bf, a, n, n_segs, ws.bits, ws.seg_counts);
    prof4_.end();
    RPT_LAUNCHED("probe_bits_kernel<lds>");
  } else {
    // PARTITIONED: the key column, tiles of slice_count(L) slices. BUCKETED: level 1 first, then the
    // same pipeline over the level-2 hash array (tiles of 128 slices, bucket by bucket), then level 1's
    // unpermute.
    const bool buck = strategy == RPT_PROBE_BUCKETED;
    uint32_t tile_slices = slice_count(L), grid_slices = tile_slices;
    uint64_t n_tiles = ceil_div(n, rpt::kTileRows), n_part = n;
    rpt::KeyArgs pa = a;
    int p_type = col->key_type;
    bool p_dense = dense;
    const uint32_t* bucket_tiles = nullptr;
    const uint32_t* dev_n_tiles = nullptr;
    uint64_t* part_bits = ws.bits;
    uint32_t* part_counts = ws.seg_counts;
    if (buck) {
      const BucketLevel1 l1{ws.counts_tm, ws.pre_bm, ws.pre_tm, ws.totals, ws.bucket_tiles, ws.bbase, ws.hashes, ws.pos1};
      int st1 = run_bucket_level1(s, col->key_type, a, dense, n, L, l1, nullptr);
      if (st1 != RPT_OK) return st1;
      tile_slices = rpt::kBucketSlices;
      grid_slices = bucket_count(L) * rpt::kBucketSlices;
      n_tiles = level2_tiles_max(n, L);
      n_part = n_tiles * rpt::kTileRows;
      pa = rpt::KeyArgs{ws.hashes, nullptr, nullptr, nullptr};
      p_type = RPT_KEY_HASH;
      p_dense = true;
      bucket_tiles = ws.bucket_tiles;
      dev_n_tiles = ws.bucket_tiles + bucket_count(L);
      part_bits = ws.bits2;
      part_counts = nullptr;
    }
    const int cus = num_cus(bf->device);
    ProfScope prof5_("partition_kernel", s);
    RPT_DISPATCH_KD(launch_partition_t, p_type, p_dense, static_cast<unsigned>(n_tiles), s, pa, n_part, tile_slices - 1,
                    n_tiles, ws.recs, ws.pos, ws.runs_tm, static_cast<int64_t*>(nullptr), dev_n_tiles);
    prof5_.end();
    RPT_LAUNCHED("partition_kernel");
    int st2 = transpose_u32(s, ws.runs_tm, n_tiles, tile_slices, ws.runs);
    if (st2 != RPT_OK) return st2;
    // exactly one resident round of slice workgroups (LDS decides how many fit per CU), never more
    // splits than tiles
    const uint64_t slice_lds = rpt::kSliceWords * 8 + 8ULL * rpt::kRotMasks;
    const uint64_t per_cu = std::max<uint64_t>(1, (160ULL << 10) / slice_lds);
    const uint64_t resident = static_cast<uint64_t>(cus) * per_cu;
    const uint32_t splits = static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>(n_tiles, resident / grid_slices)));
    const uint32_t n_items = grid_slices * splits;
    ProfScope prof6_("slice_probe_kernel", s);
    hipLaunchKernelGGL(rpt::slice_probe_kernel, dim3(static_cast<unsigned>(std::min<uint64_t>(n_items, resident))),
                       dim3(rpt::kSliceThreads), 0, s, bf->words, splits, n_tiles, ws.recs, ws.runs, ws.passb, tile_slices,
                       bucket_tiles, n_items);
    prof6_.end();
    RPT_LAUNCHED("slice_probe_kernel");
    ProfScope prof7_("unpermute_kernel", s);
    const uint64_t cap = rpt::tile_cap_for(tile_slices);
    hipLaunchKernelGGL(rpt::unpermute_kernel, dim3(static_cast<unsigned>(n_tiles)), dim3(rpt::kUnpermuteThreads), cap / 8, s,
                       ws.pos, ws.passb, n_part, cap, part_bits, part_counts, dev_n_tiles);
    prof7_.end();
    RPT_LAUNCHED("unpermute_kernel");
    if (buck) {
      ProfScope prof8b_("bucket_unpermute_kernel", s);
      hipLaunchKernelGGL(rpt::bucket_unpermute_kernel, dim3(static_cast<unsigned>(ceil_div(n, rpt::kTileRows))),
                         dim3(rpt::kBucketUnpermuteThreads), 0, s, ws.pos1, ws.bits2, n, bucket_count(L) - 1,
                         ws.counts_tm, ws.pre_tm, ws.bbase, ws.bits, ws.seg_counts);
      prof8b_.end();
      RPT_LAUNCHED("bucket_unpermute_kernel");
    }
  }
  return RPT_OK;
}

int rpt_bf_probe_phase2(const rpt_bf* bf, const uint32_t* row_sel, uint64_t n, uint32_t* out_sel,
                        uint64_t* out_count_dev, void* workspace, size_t workspace_bytes, rpt_stream_t stream) {
  if (!bf || !out_count_dev) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  if (n >= (1ULL << 32)) return fail(RPT_ERR_INVALID_ARGUMENT, "n=%llu rows exceeds uint32 sel_t", (unsigned long long)n);
  RPT_ON_DEVICE(bf->device);
  hipStream_t s = as_stream(stream);
  if (n == 0) {  // bloom_filter.cpp:63-65
    RPT_HIP(hipMemsetAsync(out_count_dev, 0, sizeof(uint64_t), s));
    return RPT_OK;
  }
  if (!out_sel) return fail(RPT_ERR_INVALID_ARGUMENT, "null out_sel");
  const int L = bf->log_num_blocks;
  const int strategy = resolve_strategy(bf->probe_strategy.load(), L, n);
  const size_t need = workspace_layout(n, L, strategy, nullptr, nullptr);
  if (!workspace || workspace_bytes < need)
    return fail(RPT_ERR_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes, need);
  ProbeWorkspace ws;
  workspace_layout(n, L, strategy, workspace, &ws);
  const uint64_t n_segs = ceil_div(n, rpt::kSegRows);
  const uint64_t n_groups = ceil_div(n_segs, rpt::kGroupSegs);
  ProfScope prof8_("group_sum_kernel", s);
  hipLaunchKernelGGL(rpt::group_sum_kernel, dim3(static_cast<unsigned>(n_groups)), dim3(rpt::kBlockThreads), 0, s,
                     ws.seg_counts, n_segs, ws.group_sums);
  prof8_.end();
  RPT_LAUNCHED("group_sum_kernel");
  ProfScope prof9_("group_scan_kernel", s);
  hipLaunchKernelGGL(rpt::group_scan_kernel, dim3(1), dim3(1024), 0, s, ws.group_sums,
                     static_cast<uint32_t>(n_groups), ws.group_offs, out_count_dev);
  prof9_.end();
  RPT_LAUNCHED("group_scan_kernel");
  ProfScope prof10_("compact_kernel", s);
  hipLaunchKernelGGL(rpt::compact_kernel, dim3(static_cast<unsigned>(n_groups)), dim3(rpt::kBlockThreads), 0, s,
                     ws.bits, ws.seg_counts, n_segs, ws.group_offs, row_sel, out_sel);
  prof10_.end();
  RPT_LAUNCHED("compact_kernel");
  return RPT_OK;
}

int rpt_bf_probe(const rpt_bf* bf, const rpt_key_column* col, const uint32_t* row_sel, uint64_t n,
                 uint32_t* out_sel, uint64_t* out_count_dev, void* workspace, size_t workspace_bytes,
                 rpt_stream_t stream) {
  if (!bf || !out_count_dev) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  RPT_ON_DEVICE(bf->device);
  int st = rpt_bf_probe_phase1(bf, col, row_sel, n, workspace, workspace_bytes, stream);
  if (st != RPT_OK) return st;
  return rpt_bf_probe_phase2(bf, row_sel, n, out_sel, out_count_dev, workspace, workspace_bytes, stream);
}


int rpt_hash_combine(const rpt_key_column* col, uint64_t n, uint64_t* inout_hashes, rpt_stream_t stream) {
  return launch_hash<true>(col, n, inout_hashes, stream);
}

int rpt_hash_keys(const rpt_key_column* col, uint64_t n, uint64_t* out_hashes, rpt_stream_t stream) {
  return launch_hash<false>(col, n, out_hashes, stream);
}

int rpt_words_or_slices(uint64_t* dst, const uint64_t* srcs, uint32_t k, uint64_t n_words, rpt_stream_t stream) {
  if (!dst || (!srcs && k > 0)) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  if (n_words == 0) return RPT_OK;
  const unsigned grid = static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(n_words / 2, rpt::kBlockThreads), 8192)));
  ProfScope prof12_("or_slices_kernel", as_stream(stream));
  hipLaunchKernelGGL(rpt::or_slices_kernel, dim3(grid), dim3(rpt::kBlockThreads), 0, as_stream(stream), dst, srcs, k,
                     n_words, 0);
  prof12_.end();
  RPT_LAUNCHED("or_slices_kernel");
  return RPT_OK;
}

int rpt_words_or(uint64_t* dst, const uint64_t* src, uint64_t n_words, rpt_stream_t stream) {
  if (!dst || !src) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  if (n_words == 0) return RPT_OK;
  const unsigned grid = static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(n_words / 2, rpt::kBlockThreads), 8192)));
  ProfScope prof13_("or_slices_kernel", as_stream(stream));
  hipLaunchKernelGGL(rpt::or_slices_kernel, dim3(grid), dim3(rpt::kBlockThreads), 0, as_stream(stream), dst, src, 1u,
                     n_words, 1);
  prof13_.end();
  RPT_LAUNCHED("or_slices_kernel");
  return RPT_OK;
}

int rpt_bf_merge_or(rpt_bf* dst, const rpt_bf* src, rpt_stream_t stream) {
  if (!dst || !src) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  if (dst->log_num_blocks != src->log_num_blocks || dst->device != src->device)
    return fail(RPT_ERR_SHAPE_MISMATCH, "merge of log_num_blocks %d (dev %d) with %d (dev %d)", dst->log_num_blocks,
                dst->device, src->log_num_blocks, src->device);
  RPT_ON_DEVICE(dst->device);
  int st = rpt_words_or(dst->words, src->words, 1ULL << dst->log_num_blocks, stream);
  if (st != RPT_OK) return st;
  hipLaunchKernelGGL(stats_merge_kernel, dim3(1), dim3(1), 0, as_stream(stream), dst->stats, src->stats);
  RPT_LAUNCHED("stats_merge_kernel");
  if (src->has_data.load()) dst->has_data.store(1);
  return RPT_OK;
}

int rpt_bf_count_bits(const rpt_bf* bf, uint64_t* out) {
  if (!bf || !out) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  RPT_ON_DEVICE(bf->device);
  unsigned long long* d = nullptr;
  RPT_HIP(hipMalloc(&d, sizeof(unsigned long long)));
  hipError_t e = hipMemset(d, 0, sizeof(unsigned long long));
  const uint64_t nw = 1ULL << bf->log_num_blocks;
  const unsigned grid = static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(nw, rpt::kBlockThreads), 4096)));
  if (e == hipSuccess) {
    hipLaunchKernelGGL(rpt::popcount_kernel, dim3(grid), dim3(rpt::kBlockThreads), 0, nullptr, bf->words, nw, d);
    e = hipGetLastError();
  }
  unsigned long long h = 0;
  if (e == hipSuccess) e = hipMemcpy(&h, d, sizeof h, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(RPT_ERR_HIP, "count_bits: %s", hipGetErrorString(e));
  *out = h;
  return RPT_OK;
}

int rpt_bf_fold(rpt_bf* bf, int* out_new_log_num_blocks) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  RPT_ON_DEVICE(bf->device);
  RPT_HIP(hipDeviceSynchronize());
  constexpr int kMinLog = 4;  // bloom_filter.h Fold: log_num_blocks_min
  for (;;) {
    if (bf->log_num_blocks <= kMinLog) break;
    uint64_t set = 0;
    int st = rpt_bf_count_bits(bf, &set);
    if (st != RPT_OK) return st;
    const uint64_t nb = 1ULL << bf->log_num_blocks;
    const uint64_t num_bits = nb * 64;
    if (4 * set >= num_bits) break;
    int folds = 1;
    while ((bf->log_num_blocks - folds) > kMinLog && (4 * set) < (num_bits >> folds)) ++folds;
    const uint64_t slice = nb >> folds;
    // target slice 0 accumulates slices 1 .. 2^folds-1 (they never overlap the target)
    const unsigned grid = static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(slice / 2, rpt::kBlockThreads), 8192)));
    ProfScope prof14_("or_slices_kernel(fold)", nullptr);
    hipLaunchKernelGGL(rpt::or_slices_kernel, dim3(grid), dim3(rpt::kBlockThreads), 0, nullptr, bf->words,
                       bf->words + slice, static_cast<uint32_t>((1u << folds) - 1), slice, 1);
    prof14_.end();
    RPT_LAUNCHED("or_slices_kernel(fold)");
    RPT_HIP(hipDeviceSynchronize());
    bf->log_num_blocks -= folds;
  }
  if (out_new_log_num_blocks) *out_new_log_num_blocks = bf->log_num_blocks;
  return RPT_OK;
}

int rpt_bf_export_words(const rpt_bf* bf, uint64_t* host_words, uint64_t n_words) {
  if (!bf || !host_words) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  if (n_words != (1ULL << bf->log_num_blocks))
    return fail(RPT_ERR_SHAPE_MISMATCH, "export of %llu words from a %llu-word filter", (unsigned long long)n_words,
                (unsigned long long)(1ULL << bf->log_num_blocks));
  RPT_ON_DEVICE(bf->device);
  RPT_HIP(hipDeviceSynchronize());
  RPT_HIP(hipMemcpy(host_words, bf->words, n_words * 8, hipMemcpyDeviceToHost));
  return RPT_OK;
}

int rpt_bf_import_words(rpt_bf* bf, const uint64_t* host_words, uint64_t n_words) {
  if (!bf || !host_words) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  if (n_words != (1ULL << bf->log_num_blocks))
    return fail(RPT_ERR_SHAPE_MISMATCH, "import of %llu words into a %llu-word filter", (unsigned long long)n_words,
                (unsigned long long)(1ULL << bf->log_num_blocks));
  RPT_ON_DEVICE(bf->device);
  RPT_HIP(hipDeviceSynchronize());
  RPT_HIP(hipMemcpy(bf->words, host_words, n_words * 8, hipMemcpyHostToDevice));
  int any = 0;
  for (uint64_t i = 0; i < n_words && !any; i++) any = host_words[i] != 0;
  bf->has_data.store(any);
  return RPT_OK;
}

int rpt_bf_copy_words_to(const rpt_bf* bf, uint64_t* dst_dev, uint64_t n_words, rpt_stream_t stream) {
  if (!bf || !dst_dev) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  if (n_words != (1ULL << bf->log_num_blocks))
    return fail(RPT_ERR_SHAPE_MISMATCH, "copy of %llu words from a %llu-word filter", (unsigned long long)n_words,
                (unsigned long long)(1ULL << bf->log_num_blocks));
  RPT_ON_DEVICE(bf->device);
  RPT_HIP(hipMemcpyAsync(dst_dev, bf->words, n_words * 8, hipMemcpyDeviceToDevice, as_stream(stream)));
  return RPT_OK;
}

int rpt_bf_copy_words_from(rpt_bf* bf, const uint64_t* src_dev, uint64_t n_words, rpt_stream_t stream) {
  if (!bf || !src_dev) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  if (n_words != (1ULL << bf->log_num_blocks))
    return fail(RPT_ERR_SHAPE_MISMATCH, "copy of %llu words into a %llu-word filter", (unsigned long long)n_words,
                (unsigned long long)(1ULL << bf->log_num_blocks));
  RPT_ON_DEVICE(bf->device);
  RPT_HIP(hipMemcpyAsync(bf->words, src_dev, n_words * 8, hipMemcpyDeviceToDevice, as_stream(stream)));
  return RPT_OK;
}


int rpt_profiling_enable(int enable) {
  g_prof_enabled.store(enable ? 1 : 0);
  return RPT_OK;
}

int rpt_profiling_reset(void) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  for (auto& r : g_prof_pending) {
    (void)hipEventSynchronize(r.end);
    g_prof_free.push_back(r.start);
    g_prof_free.push_back(r.end);
  }
  g_prof_pending.clear();
  g_prof_stats.clear();
  return RPT_OK;
}

int rpt_profiling_read(rpt_kernel_stat* out, int capacity) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  for (auto& r : g_prof_pending) {
    float ms = 0.f;
    if (hipEventSynchronize(r.end) != hipSuccess || hipEventElapsedTime(&ms, r.start, r.end) != hipSuccess)
      return -fail(RPT_ERR_HIP, "profiling: event query failed");
    auto it = std::find_if(g_prof_stats.begin(), g_prof_stats.end(), [&](const auto& p) { return p.first == r.name; });
    if (it == g_prof_stats.end()) {
      g_prof_stats.push_back({std::string(r.name), ProfStat{}});
      it = g_prof_stats.end() - 1;
    }
    it->second.launches++;
    it->second.total_ms += ms;
    g_prof_free.push_back(r.start);
    g_prof_free.push_back(r.end);
  }
  g_prof_pending.clear();
  const int n = static_cast<int>(g_prof_stats.size());
  for (int i = 0; i < n && i < capacity && out; i++) {
    memset(out[i].name, 0, sizeof out[i].name);
    strncpy(out[i].name, g_prof_stats[i].first.c_str(), sizeof out[i].name - 1);
    out[i].launches = g_prof_stats[i].second.launches;
    out[i].total_ms = g_prof_stats[i].second.total_ms;
  }
  return n;
}

// ---- bench / test workload generators (include/rpt_gpu_synth.h) ---------------------------------
int rpt_synth_build_keys(int64_t* out, uint64_t start, uint64_t n, rpt_stream_t stream) {
  if (!out) return fail(RPT_ERR_INVALID_ARGUMENT, "null out");
  if (n == 0) return RPT_OK;
  const unsigned grid = static_cast<unsigned>(std::min<uint64_t>(ceil_div(n, rpt::kBlockThreads), 8192));
  ProfScope prof15_("synth_build_kernel", as_stream(stream));
  hipLaunchKernelGGL(rpt::synth_build_kernel, dim3(grid), dim3(rpt::kBlockThreads), 0, as_stream(stream), out, start, n);
  prof15_.end();
  RPT_LAUNCHED("synth_build_kernel");
  return RPT_OK;
}

int rpt_synth_probe_keys(int64_t* out, uint64_t n_build, uint32_t p_permille, uint64_t start, uint64_t n,
                         rpt_stream_t stream) {
  if (!out) return fail(RPT_ERR_INVALID_ARGUMENT, "null out");
  if (p_permille > 1000) return fail(RPT_ERR_INVALID_ARGUMENT, "p_permille %u > 1000", p_permille);
  if (n == 0) return RPT_OK;
  const unsigned grid = static_cast<unsigned>(std::min<uint64_t>(ceil_div(n, rpt::kBlockThreads), 8192));
  ProfScope prof16_("synth_probe_kernel", as_stream(stream));
  hipLaunchKernelGGL(rpt::synth_probe_kernel, dim3(grid), dim3(rpt::kBlockThreads), 0, as_stream(stream), out, n_build,
                     p_permille, start, n);
  prof16_.end();
  RPT_LAUNCHED("synth_probe_kernel");
  return RPT_OK;
}

}  // extern "C"
