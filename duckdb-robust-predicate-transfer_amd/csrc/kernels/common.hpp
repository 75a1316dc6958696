// common.hpp — launch constants, key-column access (load_hashes) and min/max helpers.
// Part of librpt_gpu.so: included by rpt_gpu.hip (one translation unit: kernels and their launches
// stay together without relocatable device code).
#pragma once

// Measurement-only macros (RPT_EXP_*) make kernels skip work, i.e. return WRONG results: they exist for
// the A/B variants tools/build_variants.sh builds under other names (build/variants/). The product build
// (Makefile: RPT_PRODUCT_BUILD, which HIPFLAGS cannot drop) refuses them.
#if defined(RPT_PRODUCT_BUILD) && (defined(RPT_EXP_PART_STOP) || defined(RPT_EXP_SCATTER_SKIP) || \
                                   defined(RPT_EXP_STORE_SKIP_ZERO) || defined(RPT_EXP_NO_PASS_WRITE) || \
                                   defined(RPT_EXP_PROBE_NO_LDS) || defined(RPT_EXP_PROBE_NO_HASH))
#error "RPT_EXP_* measurement macros are not allowed in the product build (use tools/build_variants.sh)"
#endif

namespace rpt {

constexpr int kBlockThreads = 256;
constexpr int kWavesPerBlock = kBlockThreads / 64;
constexpr uint64_t kSegRows = 512;                 // rows per wave segment (8 per lane)
constexpr uint64_t kWordsPerSeg = kSegRows / 64;   // result-bit words per segment
constexpr uint64_t kGroupSegs = 256;               // segments per scan group (one compaction workgroup)
constexpr int kBlocksPerCU = 8;

// Partitioned ("routed") probe: the filter is cut into 128 KiB slices that fit in LDS; probe rows are
// bucketed by slice per 16 Ki- (or 32 Ki-) row tile so that every filter access is an LDS read.
#ifndef RPT_SLICE_LOG
#define RPT_SLICE_LOG 14
#endif
constexpr int kSliceLog = RPT_SLICE_LOG;               // 2^13 blocks = 64 KiB (or 2^14 = 128 KiB) per slice
constexpr uint64_t kSliceWords = 1ULL << kSliceLog;
constexpr int kMaxSliceCount = 1024;                   // P <= 1024 slices (filters <= 128 MiB at 128 KiB slices)
constexpr uint64_t kTileRows = 16384;                  // rows per partition tile (x tile_mult for large P)
// Runs are padded to kRunPad records so a lane owns kRunPad aligned records of one run and its pass
// results form one byte of bits. Tile capacity is a multiple of 128 so the tile's pass bits are
// whole 16-byte vectors.
constexpr uint32_t kRunPad = 8;
// Runs start at multiples of kRunAlign records (a multiple of kRunPad; tuning: RPT_RUN_ALIGN).
#ifndef RPT_RUN_ALIGN
#define RPT_RUN_ALIGN 8
#endif
constexpr uint32_t kRunAlign = RPT_RUN_ALIGN;
static_assert(kRunAlign % kRunPad == 0, "runs start at lane boundaries");
__host__ __device__ constexpr uint32_t pad_run(uint32_t c) { return (c + kRunAlign - 1) & ~(kRunAlign - 1); }
// Tiles of tm * kTileRows rows (tm = 1 or 2).
__host__ __device__ constexpr uint64_t tile_cap_for(uint32_t n_slices, uint32_t tm = 1) {
  return (kTileRows * tm + static_cast<uint64_t>(kRunAlign) * n_slices + 127) & ~127ULL;
}
// The plain partitioned strategy doubles its tiles above 128 slices (filters > 16 MiB): a tile's run
// per slice would otherwise average under 64 records and the slice probe's reads fragment. Measured
// (probe ms per 1e9 keys, 16 Ki -> 32 Ki rows): 1024 slices 6.25 -> 5.12, 512 slices 5.05 -> 4.6,
// 256 slices 4.31 -> 4.30 (build 0.26 -> 0.22 ms), 128 slices 3.95 -> 4.22 (one workgroup per CU
// costs the partition more than the longer runs save). The bucketed strategy's level 2 (256 slices
// per bucket) keeps tm = 1.
__host__ __device__ constexpr uint32_t tile_mult(uint32_t n_slices) { return n_slices > 128 ? 2u : 1u; }
// Bucketed strategy (filters > 128 MiB): 32 MiB buckets of 256 slices, at most 512 buckets (16 GiB).
// Bucket size (C5 probe / build ms per 1e9 keys, 8 GiB filter; level-2 tiles of 16 Ki rows): 128 slices
// 10.5 / 12.3, 256 slices 9.8 / 11.7, 512 slices 10.5 / 12.3, 1024 slices 11.0 / 12.5 -- longer level-1
// runs (a faster scatter and unpermute) against shorter level-2 runs (a slower partition and slice probe).
#ifndef RPT_BUCKET_SLICE_LOG
#define RPT_BUCKET_SLICE_LOG 8
#endif
constexpr int kBucketSliceLog = RPT_BUCKET_SLICE_LOG;
constexpr int kMaxBucketedLog = 31;  // 16 GiB
constexpr uint32_t kBucketSlices = 1u << kBucketSliceLog;
constexpr uint32_t kMaxBuckets = 512;  // 16 GiB / 32 MiB
constexpr int kTileThreads = 1024;                     // 16 waves
constexpr int kRowsPerThread = static_cast<int>(kTileRows / kTileThreads);
constexpr int kSegsPerWaveA = kRowsPerThread / 8;      // 512-row segments per wave (bucketed level 2 / build)
// Level-1 tiles of the bucketed strategy (bucket_scatter / bucket_unpermute): 16 Ki rows, independent of
// the partition tile (the scatter stages 7 B per row in LDS).
#ifndef RPT_L1_TILE_ROWS
#define RPT_L1_TILE_ROWS 16384
#endif
constexpr uint64_t kL1TileRows = RPT_L1_TILE_ROWS;
constexpr int kL1SegsPerWave = static_cast<int>(kL1TileRows / kTileThreads / 8);
// The level-2 hash array is allocated in chunks of 4 Ki rows (bucketed.hpp); a level-2 tile is 4 chunks
// of one bucket, so a 512-row segment never straddles two chunks.
constexpr int kChunkLog = 12;
constexpr uint64_t kChunkRows = 1ULL << kChunkLog;
constexpr uint32_t kChunksPerTile = static_cast<uint32_t>(kTileRows / kChunkRows);
static_assert(kChunkRows % kSegRows == 0 && kTileRows % kChunkRows == 0, "chunks hold whole segments, tiles whole chunks");
constexpr int kSliceThreads = 1024;                    // slice-probe workgroup (16 waves)
constexpr int kLdsDirectMaxLog = 14;                   // filters <= 128 KiB: whole filter in LDS
constexpr int kLdsProbeThreads = 1024;                 // whole-filter LDS probe workgroup (16 waves)
#ifndef RPT_PARTITION_SMALL_P
#define RPT_PARTITION_SMALL_P 1                        // partition of <= 4-slice filters: wave-aggregated counters
#endif
#ifndef RPT_VALU_INTERLEAVE
#define RPT_VALU_INTERLEAVE 1                          // store_segment_bits: bit interleave on VALU (lanes 0-7)
#endif
#ifndef RPT_SEL_BALLOT_EXPAND
#define RPT_SEL_BALLOT_EXPAND 1                        // dense selection vectors written 64 rows at a time, contiguously
#endif
#ifndef RPT_SEL_BALLOT_MIN
#define RPT_SEL_BALLOT_MIN 192                         // ... from this many survivors per 512 rows (unpermute_sel)
#endif
#ifndef RPT_COMPACT_BALLOT_MIN
#define RPT_COMPACT_BALLOT_MIN 384                     // ... per 512 rows in compact_kernel (its sparse path stages in LDS)
#endif
#ifndef RPT_SLICE_UNROLL
#define RPT_SLICE_UNROLL 4                             // 512-record steps in flight per wave
#endif
#ifndef RPT_PARTITION_MIN_WAVES
#define RPT_PARTITION_MIN_WAVES 8                      // 2 partition workgroups per CU (64 VGPRs) at tm = 1
#endif

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Streamed-once loads, non-temporal where it measured faster (C2 / C5 A/B, tools/ab_cfgs.sh):
// key columns in the 16 Ki-row partition and the bucketed level-1 count (partition 2.27 -> 2.16 ms,
// bucket count 1.28 -> 1.20 ms per 1e9 keys); NOT in the 32 Ki-row partition (2.62 -> 3.07 ms) nor for
// the routing intermediates (slice probe records: 0.93 -> 1.20 ms).
#ifndef RPT_NT_KEY_LOADS
#define RPT_NT_KEY_LOADS 1
#endif
#ifndef RPT_NT_REC_LOADS
#define RPT_NT_REC_LOADS 0
#endif
#ifndef RPT_NT_SLICE_LOADS
#define RPT_NT_SLICE_LOADS 1  // the persistent slice probe's prefetch of the next slice's filter words (C5 slice probe 2.58 -> 2.46 ms)
#endif
template <bool NT, typename T>
__device__ __forceinline__ T stream_load(const T* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

struct KeyArgs {
  const void* keys;
  const uint32_t* key_sel;
  const uint64_t* validity;
  const uint32_t* row_sel;
  const uint8_t* hi8 = nullptr;  // kKeySplit only: hash bits 32..39 per row
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
// MM over a full NULL-free segment of the batched loads (the bucketed level-1 scatter of a build): a
// tournament over the lane's 8 values instead of a guarded min and max per value (VGPRs 111 -> 86): C5
// build 7.58-7.65 -> 7.43-7.50 ms on one box (profiles/r04/ab_mm_tournament.txt).
#ifndef RPT_MM_TOURNAMENT
#define RPT_MM_TOURNAMENT 1
#endif
template <int K, bool DENSE, bool MM = false, bool NT = false, bool BATCH = false>
__device__ __forceinline__ void load_hashes(const KeyArgs& a, uint64_t base, uint64_t n, uint32_t lane,
                                            uint64_t (&h)[8], bool (&ok)[8], int64_t* mm = nullptr) {
  using Tr = KeyTraits<K>;
  using T = typename Tr::T;
  // rows left from `base` (uniform), so per-row bounds checks are 32-bit and addresses are
  // uniform-base + 32-bit lane offset
  const uint32_t rem = n > base ? static_cast<uint32_t>(n - base < kSegRows ? n - base : kSegRows) : 0u;
  if constexpr (DENSE && BATCH) {
    constexpr int V = Tr::kVec;
    constexpr int C = 8 / V;
    const T* kb = static_cast<const T*>(a.keys) + base;
    const uint64_t* vb = a.validity ? a.validity + (base >> 6) : nullptr;  // base is a multiple of 512
    [[maybe_unused]] const uint8_t* hb = K == kKeySplit ? a.hi8 + base : nullptr;
    T v[8];
    uint32_t vbits[C], hi4[C];  // validity bits of the lane's V rows (bits 0..V-1); kKeySplit hash bits 32..39
    if (rem == static_cast<uint32_t>(kSegRows)) {
      // A full segment (uniform branch): every load is issued back to back (with one per-lane "full
      // vector or tail" branch per 16-B load, both paths write the same registers and the compiler
      // waits for each load before issuing the next). Measured: bucketed level-1 scatter (one
      // workgroup per CU) 3.55 -> 3.38 ms; the partition and count kernels 1-3 % slower, so they keep
      // the per-load form.
#pragma unroll
      for (int c = 0; c < C; c++) {
        const uint32_t off = static_cast<uint32_t>(c * 64 * V) + lane * V;
        if constexpr (V == 2) {
          const u64x2 x = stream_load<NT>(reinterpret_cast<const u64x2*>(kb + off));
          v[c * 2] = static_cast<T>(x[0]);
          v[c * 2 + 1] = static_cast<T>(x[1]);
        } else {
          const u32x4 x = stream_load<NT>(reinterpret_cast<const u32x4*>(kb + off));
#pragma unroll
          for (int e = 0; e < V; e++) v[c * V + e] = static_cast<T>(x[e]);
        }
        hi4[c] = 0;
        if constexpr (K == kKeySplit) hi4[c] = *reinterpret_cast<const uint32_t*>(hb + off);
        vbits[c] = (1u << V) - 1;
      }
      if (Tr::kValues && vb != nullptr) {
#pragma unroll
        for (int c = 0; c < C; c++) {
          const uint32_t off = static_cast<uint32_t>(c * 64 * V) + lane * V;
          vbits[c] = static_cast<uint32_t>(vb[off >> 6] >> (off & 63));  // V | 64: one word
        }
      }
    } else {
#pragma unroll
      for (int c = 0; c < C; c++) {
        const uint32_t off = static_cast<uint32_t>(c * 64 * V) + lane * V;
#pragma unroll
        for (int e = 0; e < V; e++) v[c * V + e] = (off + e < rem) ? kb[off + e] : T(0);
        vbits[c] = (1u << V) - 1;
        if (Tr::kValues && vb != nullptr && off < rem) vbits[c] = static_cast<uint32_t>(vb[off >> 6] >> (off & 63));
        hi4[c] = 0;
        if constexpr (K == kKeySplit)
          for (int e = 0; e < V; e++) hi4[c] |= (off + e < rem ? static_cast<uint32_t>(hb[off + e]) : 0u) << (8 * e);
      }
    }
#pragma unroll
    for (int c = 0; c < C; c++) {
      const uint32_t off = static_cast<uint32_t>(c * 64 * V) + lane * V;
#pragma unroll
      for (int e = 0; e < V; e++) {
        ok[c * V + e] = off + e < rem;
        uint64_t hv = Tr::hash(v[c * V + e]);
        if constexpr (K == kKeySplit) hv |= static_cast<uint64_t>((hi4[c] >> (8 * e)) & 0xFFu) << 32;
        if (Tr::kValues && !((vbits[c] >> e) & 1u)) hv = kNullHash;
        h[c * V + e] = hv;
        if constexpr (MM && Tr::kValues && !RPT_MM_TOURNAMENT) {
          if (off + e < rem && ((vbits[c] >> e) & 1u)) {
            mm[0] = min(mm[0], static_cast<int64_t>(v[c * V + e]));
            mm[1] = max(mm[1], static_cast<int64_t>(v[c * V + e]));
          }
        }
      }
    }
    if constexpr (MM && Tr::kValues && RPT_MM_TOURNAMENT) {
      if (rem == static_cast<uint32_t>(kSegRows) && vb == nullptr) {
        // a full segment without NULLs (uniform): the 8 values' min and max by a tournament (one compare
        // per pair yields both, then 3 + 3), instead of a guarded min and max per value
        int64_t lo[4], hi[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int64_t x = static_cast<int64_t>(v[2 * q]), y = static_cast<int64_t>(v[2 * q + 1]);
          const bool lt = x < y;
          lo[q] = lt ? x : y;
          hi[q] = lt ? y : x;
        }
        mm[0] = min(mm[0], min(min(lo[0], lo[1]), min(lo[2], lo[3])));
        mm[1] = max(mm[1], max(max(hi[0], hi[1]), max(hi[2], hi[3])));
      } else {
#pragma unroll
        for (int c = 0; c < C; c++) {
          const uint32_t off = static_cast<uint32_t>(c * 64 * V) + lane * V;
#pragma unroll
          for (int e = 0; e < V; e++) {
            if (off + e < rem && ((vbits[c] >> e) & 1u)) {
              mm[0] = min(mm[0], static_cast<int64_t>(v[c * V + e]));
              mm[1] = max(mm[1], static_cast<int64_t>(v[c * V + e]));
            }
          }
        }
      }
    }
  } else if constexpr (DENSE) {
    constexpr int V = Tr::kVec;
    const T* kb = static_cast<const T*>(a.keys) + base;
    const uint64_t* vb = a.validity ? a.validity + (base >> 6) : nullptr;  // base is a multiple of 512
#pragma unroll
    for (int c = 0; c < 8 / V; c++) {
      const uint32_t off = static_cast<uint32_t>(c * 64 * V) + lane * V;
      T v[V];
      if (off + V <= rem) {
        if constexpr (V == 2) {
          const u64x2 x = stream_load<NT>(reinterpret_cast<const u64x2*>(kb + off));
          v[0] = static_cast<T>(x[0]);
          v[1] = static_cast<T>(x[1]);
        } else {
          const u32x4 x = stream_load<NT>(reinterpret_cast<const u32x4*>(kb + off));
#pragma unroll
          for (int e = 0; e < V; e++) v[e] = static_cast<T>(x[e]);
        }
      } else {
#pragma unroll
        for (int e = 0; e < V; e++) v[e] = (off + e < rem) ? kb[off + e] : T(0);
      }
      // validity bits of this lane's V rows, shifted down to bits 0..V-1 (V | 64: one word)
      uint32_t vbits = (1u << V) - 1;
      if (Tr::kValues && vb != nullptr && off < rem) vbits = static_cast<uint32_t>(vb[off >> 6] >> (off & 63));
      uint32_t hi4 = 0;  // kKeySplit: the V rows' hash bits 32..39
      if constexpr (K == kKeySplit) {
        const uint8_t* hb = a.hi8 + base;
        if (off + V <= rem) hi4 = *reinterpret_cast<const uint32_t*>(hb + off);
        else
          for (int e = 0; e < V; e++) hi4 |= (off + e < rem ? static_cast<uint32_t>(hb[off + e]) : 0u) << (8 * e);
      }
#pragma unroll
      for (int e = 0; e < V; e++) {
        ok[c * V + e] = off + e < rem;
        uint64_t hv = Tr::hash(v[e]);
        if constexpr (K == kKeySplit) hv |= static_cast<uint64_t>((hi4 >> (8 * e)) & 0xFFu) << 32;
        if (Tr::kValues && !((vbits >> e) & 1u)) hv = kNullHash;
        h[c * V + e] = hv;
        if constexpr (MM && Tr::kValues) {
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
        if constexpr (K == kKeySplit) hv |= static_cast<uint64_t>(a.hi8[k]) << 32;
        const bool valid = valid_at(a.validity, k);
        if (Tr::kValues && !valid) hv = kNullHash;
        if constexpr (MM && Tr::kValues) {
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
#ifndef RPT_DPP_MINMAX
#define RPT_DPP_MINMAX 1
#endif
// One DPP step on both 32-bit halves of an int64; lanes the row mask disables keep their own value.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ int64_t dpp_i64(int64_t v) {
  const uint64_t u = static_cast<uint64_t>(v);
  const int lo = static_cast<int>(static_cast<uint32_t>(u)), hi = static_cast<int>(static_cast<uint32_t>(u >> 32));
  const uint32_t rlo = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(lo, lo, CTRL, ROW_MASK, 0xf, false));
  const uint32_t rhi = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(hi, hi, CTRL, ROW_MASK, 0xf, false));
  return static_cast<int64_t>((static_cast<uint64_t>(rhi) << 32) | rlo);
}
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ void minmax_step(int64_t& mn, int64_t& mx) {
  mn = min(mn, dpp_i64<CTRL, ROW_MASK>(mn));
  mx = max(mx, dpp_i64<CTRL, ROW_MASK>(mx));
}
__device__ __forceinline__ void wave_minmax(int64_t& mn, int64_t& mx) {
#if RPT_DPP_MINMAX
  // quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror: every lane holds its row's value;
  // row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3): lane 63 holds the wave's. All VALU (DPP),
  // where __shfl_xor costs 24 ds_bpermute per call (the level-1 count: +0.28 ms per 1e9 build keys).
  minmax_step<0xB1, 0xf>(mn, mx);
  minmax_step<0x4E, 0xf>(mn, mx);
  minmax_step<0x141, 0xf>(mn, mx);
  minmax_step<0x140, 0xf>(mn, mx);
  minmax_step<0x142, 0xa>(mn, mx);
  minmax_step<0x143, 0xc>(mn, mx);
  auto lane63 = [](int64_t v) {
    const uint64_t u = static_cast<uint64_t>(v);
    const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(u)), 63));
    const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(u >> 32)), 63));
    return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
  };
  mn = lane63(mn);
  mx = lane63(mx);
#else
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
#endif
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
// RPT_PROBE_BUFSTORE = 1 (measured, off): a few lanes' stores (a segment's 8 result words from lanes 0-7, its count
// from lane 0) as buffer stores through a descriptor covering only those bytes, so the other lanes' stores are
// dropped by the descriptor's range check instead of being skipped by a branch. A store behind an exec-skip branch
// leaves the compiler's count of outstanding memory operations unknown at the pipelined probe loop's head, where it
// then waits for all of them (s_waitcnt vmcnt(0)). Removing that wait did not speed the probe (JOBDIM int64 probe
// 1.567-1.570 vs 1.577-1.579 ms, int32 and the gather probe unchanged, profiles/r06/ab_pipeline.txt): its skeleton
// is bound by the result words' HBM writes inside the key stream (tools/ubench/ubench_skeleton.hip). Global memory
// only (not LDS).
#ifndef RPT_PROBE_BUFSTORE
#define RPT_PROBE_BUFSTORE 0
#endif
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
constexpr int kRawBufferWord3 = 0x00020000;  // gfx9 raw buffer descriptor word 3: 32-bit data format, no swizzle
__device__ __forceinline__ void store_lanes_b64(uint64_t* base, uint32_t valid_bytes, uint32_t lane, uint64_t v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, static_cast<int>(valid_bytes), kRawBufferWord3);
  __builtin_amdgcn_raw_buffer_store_b64(u32x2{static_cast<uint32_t>(v), static_cast<uint32_t>(v >> 32)}, r,
                                        static_cast<int>(lane * 8), 0, 0);
}
__device__ __forceinline__ void store_lanes_b32(uint32_t* base, uint32_t valid_bytes, uint32_t lane, uint32_t v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, static_cast<int>(valid_bytes), kRawBufferWord3);
  __builtin_amdgcn_raw_buffer_store_b32(v, r, static_cast<int>(lane * 4), 0, 0);
}

// The 8 pass flags a lane holds for a 512-row segment, in load_hashes<K, DENSE> order -> the segment's
// row-ordered result words (8 x 64 bits, Arrow Find layout) and its survivor count. BUF: global outputs, written by
// buffer stores (store_lanes_*); seg_counts may then be null (its store covers no bytes).
template <int K, bool DENSE, bool BUF = false>
__device__ __forceinline__ void store_segment_bits(const bool (&pass)[8], uint32_t lane, uint64_t seg,
                                                   uint64_t* __restrict__ out_bits, uint32_t* __restrict__ seg_counts) {
  uint64_t word[8];
  uint32_t cnt = 0;
  if constexpr (DENSE && RPT_VALU_INTERLEAVE) {
    // lane w < 8 builds result word w from the two (V = 2) or four (V = 4) ballots it interleaves: the
    // bit spreading runs once on the vector unit instead of eight times on the scalar unit
    constexpr int V = KeyTraits<K>::kVec;
    uint64_t b[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      b[j] = ballot64(pass[j]);
      cnt += __popcll(b[j]);
    }
    const uint32_t w = lane & 7, c = w / V, q = w % V;
    uint64_t mine = 0;
#pragma unroll
    for (int e = 0; e < V; e++) {
      uint64_t src = 0;  // ballot c * V + e of this lane's word
#pragma unroll
      for (int cc = 0; cc < 8 / V; cc++) src = (c == static_cast<uint32_t>(cc)) ? b[cc * V + e] : src;
      if constexpr (V == 2) mine |= spread2(src >> (32 * q)) << e;
      else mine |= spread4(src >> (16 * q)) << e;
    }
    if constexpr (BUF) {
      store_lanes_b64(out_bits + seg * kWordsPerSeg, kWordsPerSeg * 8, lane, mine);
      store_lanes_b32(seg_counts + seg, seg_counts != nullptr ? 4u : 0u, lane, cnt);
    } else {
      if (lane < kWordsPerSeg) out_bits[seg * kWordsPerSeg + lane] = mine;
      if (seg_counts != nullptr && lane == 0) seg_counts[seg] = cnt;
    }
    return;
  } else if constexpr (DENSE) {
    constexpr int V = KeyTraits<K>::kVec;
    uint64_t b[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      b[j] = ballot64(pass[j]);
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
      word[j] = ballot64(pass[j]);
      cnt += __popcll(word[j]);
    }
  }
  uint64_t mine = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) mine = (lane == static_cast<uint32_t>(j)) ? word[j] : mine;
  if (lane < kWordsPerSeg) out_bits[seg * kWordsPerSeg + lane] = mine;
  if (seg_counts != nullptr && lane == 0) seg_counts[seg] = cnt;
}

}  // namespace rpt
