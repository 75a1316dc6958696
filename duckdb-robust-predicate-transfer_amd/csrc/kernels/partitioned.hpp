// partitioned.hpp — slice records, partition / transpose / slice probe / slice insert / unpermute.
// Part of librpt_gpu.so: included by rpt_gpu.hip (one translation unit: kernels and their launches
// stay together without relocatable device code).
#pragma once

namespace rpt {

// Inclusive wave-wide max scan of non-negative values (DPP: rows of 16, then row broadcasts 15 / 31).
__device__ __forceinline__ uint32_t wave_inclusive_max(uint32_t v) {
  v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x111, 0xf, 0xf, false)));
  v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x112, 0xf, 0xf, false)));
  v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x114, 0xf, 0xf, false)));
  v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x118, 0xf, 0xf, false)));
  v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x142, 0xa, 0xf, false)));
  v = max(v, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x143, 0xc, 0xf, false)));
  return v;
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

// Stores of the partition's outputs (records, row map). With 16 Ki-row tiles (TM = 1) they are
// non-temporal: gigabytes re-read by the next kernels from HBM anyway, and keeping them out of the
// caches helps the neighbours (C2: partition 2.26 -> 2.25 ms, slice probe 0.877 -> 0.863 ms). The
// TM = 2 copy-out (16-B pieces assembled from unpadded LDS) got much slower with them: C3 partition
// 2.59 -> 3.39 ms.
#ifndef RPT_NT_PART_STORES
#define RPT_NT_PART_STORES 1
#endif
template <bool NT, typename T>
__device__ __forceinline__ void part_store(T* p, T v) {
  if constexpr (NT && RPT_NT_PART_STORES) {
    __builtin_nontemporal_store(v, p);
  } else {
    *p = v;
  }
}

// Where pass 1 parks a row's record in LDS until pass 2 takes it back (same thread, same slot): any
// per-segment bijection works, so lane-major slots (j * 64 + lane: consecutive words across the wave,
// no bank conflicts) instead of the row's own position (stride V words across lanes: 2- / 4-way
// conflicts for int64 / int32 keys).
#ifndef RPT_PARK_LANE_MAJOR
#define RPT_PARK_LANE_MAJOR 1
#endif
template <int K, bool DENSE>
__device__ __forceinline__ uint32_t park_slot(int j, uint32_t lane) {
#if RPT_PARK_LANE_MAJOR
  return static_cast<uint32_t>(j) * 64u + lane;
#else
  return seg_row<K, DENSE>(j, lane);
#endif
}

// ---- partitioned probe, A: bucket a tile of kTileRows rows by filter slice ------------------------
// Row r of the tile gets record slice_record(hash) stored at position pos(r) of the tile's
// slice-sorted record array (runs padded to kRunPad records); pos(r) is written per row (u16) so
// the unpermute step can restore row order. Per tile the padded runs (start << 16 | length) are
// written tile-major (one coalesced 4*P-byte row); runs_transpose_kernel turns them slice-major for
// the slice kernel. Two passes over the rows held in registers: count per slice (LDS atomics), scan,
// then claim positions with an LDS cursor per slice and scatter.
// TM = 1 (16 Ki rows): the LDS copy of the tile has the padded layout of the output (tile_cap records)
// and leaves as one contiguous 16-B stream. TM = 2 (32 Ki rows, P > 128; at P = 1024 a padded copy would
// not fit in 160 KiB): the LDS copy is UNPADDED (kTileRows records) and the padding exists only in global
// memory. A record at unpadded LDS position q of slice s goes to padded position q + s_delta[s]; the
// copy-out walks the padded layout in 16-B pieces (a piece never straddles two runs: runs start at
// multiples of kRunPad) and finds each piece's slice in s_gslice (one u16 per kRunPad-record group).
// Dynamic LDS (partition_lds_bytes): records, then count / cursor [/ delta] per slice [, s_gslice].
__host__ __device__ constexpr uint64_t partition_lds_bytes(uint32_t n_slices, uint32_t tm) {
  return tm == 1 ? tile_cap_for(n_slices, 1) * 4 + 2ULL * n_slices * 4
                 : kTileRows * tm * 4 + 3ULL * n_slices * 4 + (tile_cap_for(n_slices, tm) / kRunPad) * 2;
}
// SP > 0 (filters of at most SP slices, TM = 1): 16 Ki rows land on so few LDS counters that same-address
// atomics serialize (P = 2: 4.3 ms per 1e9 rows, P = 4: 2.9 ms, P >= 8: 2.3-2.5 ms). Each lane then counts
// its rows per slice in registers, a wave adds its totals with one atomic per slice, and rows take
// positions from per-lane cursors (wave base + DPP prefix over lanes).
// NOPARK (dense keys, SP = 0; TM = 1 only for int32 keys): the records stay in registers between the passes
// instead of being parked in LDS. TM = 1: 16 VGPRs, which the int32 kernel fits within the 64 of two
// workgroups per CU (63 used; the int64 kernel does not); its partition is bound by its LDS ops, not by HBM
// (DESIGN §5): 1.84 -> 1.79 ms per 1e9 rows (profiles/r04/ab_part_nopark.txt). TM = 2 (one workgroup per CU,
// 128 VGPRs): 32 VGPRs, 115 used: C3 int32 partition 2.37 -> 2.26-2.28 ms, int64 2.64 -> 2.60-2.64, builds
// -5 % (profiles/r04/ab_part_nopark_tm2.txt).
#ifndef RPT_PART_NOPARK
#define RPT_PART_NOPARK 1
#endif
template <int K, bool DENSE, bool MM, int TM, int SP = 0>
__global__ __launch_bounds__(kTileThreads, TM == 1 ? RPT_PARTITION_MIN_WAVES : 4) void partition_kernel(
    KeyArgs a, uint64_t n, uint32_t slice_mask, uint64_t n_tiles, uint32_t* __restrict__ recs,
    uint16_t* __restrict__ pos_out, uint32_t* __restrict__ runs_tm, int64_t* __restrict__ stats,
    const uint32_t* __restrict__ dev_n_tiles, const uint32_t* __restrict__ chunk_map) {
  // dev_n_tiles (bucketed strategy): the tile count is only known on the device; the grid is an upper
  // bound and surplus workgroups leave (their run-table rows are never read).
  // chunk_map (bucketed strategy, TM = 1): tile t's rows are the kChunksPerTile chunks chunk_map[4t ..]
  // of the level-2 hash array (every row valid: the lists are padded); otherwise rows tile * kTR ...
  if (dev_n_tiles != nullptr && blockIdx.x >= *dev_n_tiles) return;
  constexpr bool PAD = TM == 1;
  constexpr uint64_t kTR = kTileRows * TM;               // rows of this tile
  constexpr int kRPT = static_cast<int>(kTR / kTileThreads), kSPW = kRPT / 8;
  constexpr bool NOPARK = RPT_PART_NOPARK && ((K == 1 && TM == 1) || TM == 2) && SP == 0 && DENSE;  // records stay in registers
  extern __shared__ uint32_t s_dyn[];
  const uint32_t n_slices = slice_mask + 1;
  const uint64_t tile_cap = tile_cap_for(n_slices, TM);
  uint32_t* s_rec = s_dyn;
  uint32_t* s_cnt = s_dyn + (PAD ? tile_cap : kTR);  // rows per slice in this tile
  uint32_t* s_cur = s_cnt + n_slices;        // run start (padded if PAD), then scatter cursor (start + count)
  uint32_t* s_delta = s_cur + n_slices;      // !PAD: padded start - unpadded start
  uint16_t* s_gslice = reinterpret_cast<uint16_t*>(s_delta + n_slices);  // slice of each kRunPad group
  __shared__ int64_t s_mm[kTileThreads / 64][2];  // MM: each wave's key min / max
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  {  // one tile per workgroup (no persistent loop: keeps per-lane invariants out of registers)
    const uint64_t tile = blockIdx.x;
    for (uint32_t i = threadIdx.x; i < n_slices; i += kTileThreads) s_cnt[i] = 0;
    __syncthreads();
    const uint64_t tile_base = tile * kTR;
    // pass 1: hash, stage the record in LDS (NOPARK: in rec[]), count rows per slice; the 16-bit slice ids
    // stay in registers (2 per word).
    static_assert(kMaxSliceCount <= 65536, "slice ids are packed as 16 bits");
    uint32_t sl2[kRPT / 2] = {};
    uint32_t rec[kRPT];  // pass 2's records (NOPARK: already pass 1's)
    [[maybe_unused]] uint32_t lc[SP > 0 ? SP : 1] = {};  // SP: this lane's rows per slice
    int64_t wmn = kMinInit, wmx = kMaxInit;  // wave-uniform: the key min/max stays out of VGPRs
#pragma unroll
    for (int sg = 0; sg < kSPW; sg++) {
      const uint32_t seg_local = wave * (kSPW * kSegRows) + sg * kSegRows;
      uint64_t hh[8];
      bool oo[8];
      int64_t mm[2] = {kMinInit, kMaxInit};
      if (chunk_map != nullptr) {
        const uint64_t src = static_cast<uint64_t>(chunk_map[tile * kChunksPerTile + (seg_local >> kChunkLog)]) * kChunkRows +
                             (seg_local & (kChunkRows - 1));
        load_hashes<K, DENSE, MM, TM == 1 && RPT_NT_KEY_LOADS>(a, src, ~0ULL, lane, hh, oo, mm);
      } else {
        load_hashes<K, DENSE, MM, TM == 1 && RPT_NT_KEY_LOADS>(a, tile_base + seg_local, n, lane, hh, oo, mm);
      }
      if constexpr (MM && KeyTraits<K>::kValues) {
        wave_minmax(mm[0], mm[1]);
        wmn = min(wmn, mm[0]);
        wmx = max(wmx, mm[1]);
      }
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const uint32_t sl = static_cast<uint32_t>(hh[j] >> (kLogNumMasks + 6 + kSliceLog)) & slice_mask;
        if constexpr (NOPARK) rec[sg * 8 + j] = slice_record(hh[j]);
        else s_rec[seg_local + park_slot<K, DENSE>(j, lane)] = slice_record(hh[j]);
        sl2[(sg * 8 + j) >> 1] |= sl << (16 * (j & 1));
        if constexpr (SP > 0) {
#pragma unroll
          for (int q = 0; q < SP; q++) lc[q] += (oo[j] && sl == static_cast<uint32_t>(q)) ? 1u : 0u;
        } else {
          if (oo[j]) atomicAdd(&s_cnt[sl], 1u);
        }
      }
    }
    if constexpr (MM && KeyTraits<K>::kValues) {  // published once per workgroup at the end
      if (lane == 0) {
        s_mm[wave][0] = wmn;
        s_mm[wave][1] = wmx;
      }
    }
    [[maybe_unused]] uint32_t lofs[SP > 0 ? SP : 1], wtot[SP > 0 ? SP : 1];
    if constexpr (SP > 0) {  // one atomic per wave and slice
#pragma unroll
      for (int q = 0; q < SP; q++) {
        const uint32_t inc = wave_inclusive_sum(lc[q]);
        lofs[q] = inc - lc[q];
        wtot[q] = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(inc), 63));
        if (lane == 0 && wtot[q] != 0) atomicAdd(&s_cnt[q], wtot[q]);
      }
    }
    __syncthreads();
    if (wave == 0) {  // exclusive scans of the slice counts, unpadded and padded to kRunPad: kMaxSliceCount/64 per lane
      constexpr int kPer = kMaxSliceCount / 64;
      uint32_t c[kPer], t = 0, tp = 0;
#pragma unroll
      for (int i = 0; i < kPer; i++) {
        const uint32_t idx = lane * kPer + i;
        c[i] = idx < n_slices ? s_cnt[idx] : 0u;
        t += c[i];
        tp += pad_run(c[i]);
      }
      uint32_t off = wave_inclusive_sum(t) - t, poff = wave_inclusive_sum(tp) - tp;
#pragma unroll
      for (int i = 0; i < kPer; i++) {
        const uint32_t idx = lane * kPer + i;
        if (idx < n_slices) {
          if constexpr (PAD) {
            s_cur[idx] = poff;
          } else {
            s_cur[idx] = off;
            s_delta[idx] = poff - off;
          }
        }
        off += c[i];
        poff += pad_run(c[i]);
      }
    }
#ifndef RPT_EXP_PART_STOP
#define RPT_EXP_PART_STOP 0  // measurement only: 1 = stop after pass 1 + the scans, 2 = after the scatter
#endif
    if (RPT_EXP_PART_STOP == 1) return;
    // pass 2: pull this thread's records back out of the row-ordered staging (NOPARK: nothing to pull) ...
#pragma unroll
    for (int sg = 0; sg < (NOPARK ? 0 : kSPW); sg++) {
      const uint32_t seg_local = wave * (kSPW * kSegRows) + sg * kSegRows;
#pragma unroll
      for (int j = 0; j < 8; j++) rec[sg * 8 + j] = s_rec[seg_local + park_slot<K, DENSE>(j, lane)];
    }
    __syncthreads();
    [[maybe_unused]] uint32_t cur[SP > 0 ? SP : 1];
    if constexpr (SP > 0) {  // this lane's first position per slice: the wave's base + earlier lanes' rows
#pragma unroll
      for (int q = 0; q < SP; q++) {
        uint32_t wb = 0;
        if (lane == 0 && wtot[q] != 0) wb = atomicAdd(&s_cur[q], wtot[q]);
        cur[q] = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(wb))) + lofs[q];
      }
    }
    // ... and scatter them to their slice-sorted (unpadded) LDS positions; the row map gets the padded one
#pragma unroll
    for (int sg = 0; sg < kSPW; sg++) {
      const uint64_t base = tile_base + wave * (kSPW * kSegRows) + sg * kSegRows;
      const uint32_t seg_rem = n > base ? static_cast<uint32_t>(n - base < kSegRows ? n - base : kSegRows) : 0u;
      uint16_t pv[8];
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const int jj = sg * 8 + j;
        const uint32_t sl = (sl2[jj >> 1] >> (16 * (jj & 1))) & 0xFFFFu;
        const bool ok = seg_row<K, DENSE>(j, lane) < seg_rem;
        uint32_t p = 0;
        if (ok) {
          uint32_t q;
          if constexpr (SP > 0) {
            q = cur[0];
#pragma unroll
            for (int t = 1; t < SP; t++) q = sl == static_cast<uint32_t>(t) ? cur[t] : q;
#pragma unroll
            for (int t = 0; t < SP; t++) cur[t] += sl == static_cast<uint32_t>(t) ? 1u : 0u;
          } else {
            q = atomicAdd(&s_cur[sl], 1u);
          }
          s_rec[q] = rec[jj];
          p = PAD ? q : q + s_delta[sl];
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
            part_store<TM == 1>(reinterpret_cast<uint32_t*>(pos_out + row0),
                       static_cast<uint32_t>(pv[c * 2]) | (static_cast<uint32_t>(pv[c * 2 + 1]) << 16));
          } else {
            part_store<TM == 1>(reinterpret_cast<uint64_t*>(pos_out + row0),
                       static_cast<uint64_t>(pv[c * 4]) | (static_cast<uint64_t>(pv[c * 4 + 1]) << 16) |
                           (static_cast<uint64_t>(pv[c * 4 + 2]) << 32) | (static_cast<uint64_t>(pv[c * 4 + 3]) << 48));
          }
        }
      } else {
#pragma unroll
        for (int c = 0; c < 8; c++) pos_out[base + c * 64 + lane] = pv[c];
      }
    }
    __syncthreads();
    if (RPT_EXP_PART_STOP == 2) return;
    // records of the tile in the padded layout, 16 B per thread and step (pad slots hold stale values:
    // probed, never read back); the scatter left s_cur[i] = start_i + count_i
    u32x4* dst = reinterpret_cast<u32x4*>(recs + tile * tile_cap);
    if constexpr (PAD) {
      const uint32_t used = s_cur[slice_mask] - s_cnt[slice_mask] + pad_run(s_cnt[slice_mask]);
      const u32x4* src = reinterpret_cast<const u32x4*>(s_rec);
      for (uint32_t i = threadIdx.x; i < used / 4; i += kTileThreads) part_store<TM == 1>(dst + i, src[i]);
      for (uint32_t i = threadIdx.x; i < n_slices; i += kTileThreads)
        runs_tm[tile * n_slices + i] = ((s_cur[i] - s_cnt[i]) << 16) | s_cnt[i];  // padded start | true count
    } else {
      // each slice owns the kRunPad-record groups of its padded run
      for (uint32_t i = threadIdx.x; i < n_slices; i += kTileThreads) {
        const uint32_t c = s_cnt[i], pst = s_cur[i] - c + s_delta[i];
        for (uint32_t g = pst / kRunPad; g < (pst + pad_run(c)) / kRunPad; g++) s_gslice[g] = static_cast<uint16_t>(i);
      }
      __syncthreads();
      const uint32_t used = s_cur[slice_mask] + s_delta[slice_mask] - s_cnt[slice_mask] + pad_run(s_cnt[slice_mask]);
      for (uint32_t i = threadIdx.x; i < used / 4; i += kTileThreads) {
        const uint32_t q = 4 * i - s_delta[s_gslice[(4 * i) / kRunPad]];  // unpadded position of the piece
        u32x4 v;
#pragma unroll
        for (int e = 0; e < 4; e++) v[e] = s_rec[min(q + e, static_cast<uint32_t>(kTR) - 1)];
        part_store<TM == 1>(dst + i, v);
      }
      for (uint32_t i = threadIdx.x; i < n_slices; i += kTileThreads)
        runs_tm[tile * n_slices + i] = ((s_cur[i] - s_cnt[i] + s_delta[i]) << 16) | s_cnt[i];  // padded start | true count
    }
    __syncthreads();
  }
  if constexpr (MM && KeyTraits<K>::kValues) {
    // one no-return atomic pair per workgroup (a per-wave publish with its load round trip stalled the
    // wave before pass 1's barrier); a few thousand per build, so no pre-check
    if (threadIdx.x == 0) {
      int64_t mn = kMinInit, mx = kMaxInit;
      for (int w = 0; w < kTileThreads / 64; w++) {
        mn = min(mn, s_mm[w][0]);
        mx = max(mx, s_mm[w][1]);
      }
      if (mn != kMinInit) (void)__hip_atomic_fetch_min(stats, mn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (mx != kMaxInit) (void)__hip_atomic_fetch_max(stats + 1, mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// runs_sm[slice][tile] = runs_tm[tile][slice], through 64 x 64 LDS tiles (both sides coalesced).
// heavy != nullptr: a slice with a run longer than heavy_run in any tile is stamped heavy[slice] = epoch (a probe
// key skewed onto that slice; the slice probe then gives it more work items). Stale stamps of other calls only
// change how the work is divided, never a result.
__global__ __launch_bounds__(kBlockThreads) void runs_transpose_kernel(const uint32_t* __restrict__ runs_tm,
                                                                      uint32_t n_slices, uint64_t n_tiles,
                                                                      uint32_t* __restrict__ runs_sm,
                                                                      uint32_t* __restrict__ heavy, uint32_t heavy_run,
                                                                      uint32_t epoch) {
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
    if (t < n_tiles && s0 + r < n_slices) {
      const uint32_t v = s_t[c][r];
      runs_sm[static_cast<uint64_t>(s0 + r) * n_tiles + t] = v;
      if (heavy != nullptr && (v & 0xFFFFu) > heavy_run) heavy[s0 + r] = epoch;
    }
  }
}

// ---- partitioned probe, B: one workgroup per (slice, tile range) probes its records from LDS -------

// The runs of 64 consecutive tiles are walked as ONE flattened record stream per wave: record k of
// the stream belongs to the tile whose inclusive run-length prefix first exceeds k. Runs are padded
// to kRunPad = 8 records, so each lane owns 8 consecutive, 32-byte aligned records of one run: two
// 16-B loads and one byte of pass bits per lane, 512 records per wave step. Each lane finds the run
// of its 8-record slot through a per-wave LDS window (probe_slice_runs_tbl). Record offsets are
// 32-bit relative to the batch's first tile (a uniform base pointer).
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

// Work items are dealt to workgroups round-robin, and workgroup b runs on XCD b % 8. With
// RPT_SLICE_XCD_MAP the items are renumbered so that each XCD gets a contiguous range of
// (slice, split) items. The workgroups resident on one XCD then probe adjacent slices over the same
// tiles at about the same time. Adjacent slices' runs are adjacent in each tile, so a run's partial
// first and last 128-B lines, fetched by its neighbour's workgroup, can be L2 hits instead of
// over-fetch. Needs item and grid counts divisible by the XCD count (otherwise: identity).
#ifndef RPT_SLICE_XCD_MAP
#define RPT_SLICE_XCD_MAP 1
#endif
constexpr uint32_t kXcds = 8;
__device__ __forceinline__ uint32_t xcd_item(uint32_t item, uint32_t n_items) {
  if (!RPT_SLICE_XCD_MAP || n_items % kXcds != 0 || gridDim.x % kXcds != 0) return item;
  return (item % kXcds) * (n_items / kXcds) + item / kXcds;
}

// Probe the runs of tiles [sw.t_lo, sw.t_hi) of one slice held in LDS (see above).
// Tiles per wave batch: 64 (one run per lane), or fewer so that all kSliceThreads/64 waves get work.
__device__ __forceinline__ uint32_t batch_tiles(uint64_t n_t) {
  constexpr uint64_t kWaves = kSliceThreads / 64;
  return static_cast<uint32_t>(n_t >= 64 * kWaves ? 64 : (n_t + kWaves - 1) / kWaves);
}

// Same walk as probe_slice_runs, with the slot -> run lookup through a per-wave LDS window instead of
// a uniform loop over the runs a step overlaps (whose cost grows with the number of runs per step:
// ~14 at P = 1024). A slot is 8 records (kRunPad) of one run; a window is the kUnroll steps of 64
// slots a wave has in flight. Per window each non-empty run marks its first slot in the window with
// its lane + 1 (the run covering the window start marks slot 0), a max scan over the window carries
// the marks forward, and two ds_bpermutes fetch the run's base slot and stream prefix: ~15 VALU per
// step whatever the run lengths.
__device__ __forceinline__ void probe_slice_runs_tbl(const uint64_t* s_slice, const uint64_t* s_rmasks,
                                                     uint32_t* s_win, const SliceWork& sw, uint64_t n_tiles,
                                                     const uint32_t* __restrict__ recs,
                                                     const uint32_t* __restrict__ runs,
                                                     uint8_t* __restrict__ passbits, uint32_t tile_cap) {
  constexpr int kUnroll = RPT_SLICE_UNROLL;
  constexpr uint32_t kWin = 64 * kUnroll;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr uint32_t kWaves = kSliceThreads / 64;
  uint32_t* win = s_win + wave * kWin;
  const uint64_t t_lo = sw.t_lo, t_hi = sw.t_hi;
  const uint32_t* my_runs = runs + static_cast<uint64_t>(sw.run_row) * n_tiles;
  const uint32_t bt = batch_tiles(t_hi - t_lo);
  const uint32_t my = lane < bt ? lane : ~0u >> 1;  // lanes >= bt hold no run
  uint32_t info_next = (t_lo + wave * bt + my < t_hi) ? my_runs[t_lo + wave * bt + my] : 0u;
  for (uint64_t tb = t_lo + wave * bt; tb < t_hi; tb += kWaves * bt) {
    const uint32_t info = info_next;  // the next batch's runs are fetched while this one is probed
    info_next = (tb + kWaves * bt + my < t_hi) ? my_runs[tb + kWaves * bt + my] : 0u;
    const uint32_t nslot = pad_run(info & 0xFFFFu) / kRunPad;
    const uint32_t base = (lane * tile_cap + (info >> 16)) / kRunPad;  // first slot, relative to the batch
    const uint32_t* brecs = recs + tb * tile_cap;                     // uniform
    uint8_t* bpass = passbits + tb * (tile_cap / kRunPad);
    const uint32_t incl = wave_inclusive_sum(nslot);
    const uint32_t excl = incl - nslot;
    const uint32_t total = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), 63));
    const int base_m_excl = static_cast<int>(base - excl);  // slot s of this run -> base + (s - excl)
    const int real_p_excl = static_cast<int>((info & 0xFFFFu) + excl * kRunPad);  // real records left: this - 8 s
    for (uint32_t w0 = 0; w0 < total; w0 += kWin) {
#pragma unroll
      for (int u = 0; u < kUnroll; u++) win[u * 64 + lane] = 0u;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (nslot != 0 && excl < w0 + kWin && incl > w0) win[(excl > w0 ? excl : w0) - w0] = lane + 1;
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
      uint32_t off[kUnroll], keep[kUnroll];
      u32x4 rec[kUnroll][2];
      uint32_t carry = 0;
#pragma unroll
      for (int u = 0; u < kUnroll; u++) {
        const uint32_t slot = w0 + u * 64 + lane;
        uint32_t m = wave_inclusive_max(win[u * 64 + lane]);
        m = max(m, carry);
        carry = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(m), 63));
        const int src = static_cast<int>(m - 1) << 2;  // lane of the run holding this slot (byte address)
        const uint32_t rel = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, base_m_excl)) + slot;
        // pad slots get pass bit 0, so a tile's pass-bit popcount is its survivor count
        const int left = __builtin_amdgcn_ds_bpermute(src, real_p_excl) - static_cast<int>(slot * kRunPad);
        keep[u] = left >= 8 ? 0xFFu : (left > 0 ? (1u << left) - 1u : 0u);
        off[u] = slot < total ? rel * kRunPad : ~0u;
        rec[u][0] = rec[u][1] = u32x4{0, 0, 0, 0};
        if (w0 + u * 64 < total && off[u] != ~0u) {  // (first test uniform: the window's tail steps)
          rec[u][0] = stream_load<RPT_NT_REC_LOADS>(reinterpret_cast<const u32x4*>(brecs + off[u]));
          rec[u][1] = stream_load<RPT_NT_REC_LOADS>(reinterpret_cast<const u32x4*>(brecs + off[u] + 4));
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int u = 0; u < kUnroll; u++) {
        if (w0 + u * 64 >= total) break;  // uniform: a batch's last window is often part-filled
        uint32_t bits = 0;
#pragma unroll
        for (int e = 0; e < 8; e++) bits |= static_cast<uint32_t>(probe_rec(s_slice, s_rmasks, rec[u][e >> 2][e & 3])) << e;
        if (off[u] != ~0u) bpass[off[u] / kRunPad] = static_cast<uint8_t>(bits & keep[u]);
      }
    }
  }
}

// Skewed probe keys (partitioned strategy): items [0, base) are the (slice, split) items above, except that a
// heavy slice's are empty; items [base, base * (1 + mult)) split every slice mult times finer and are empty
// except for the heavy slices'. A uniform batch (no heavy slice) keeps the base items' work.
struct SkewItems {
  const uint32_t* heavy = nullptr;  // nullptr: no skew handling (n_items == base)
  uint32_t epoch = 0, base = 0, mult = 1;
};
__device__ __forceinline__ SliceWork slice_work_skew(uint32_t item, uint32_t splits, uint64_t n_tiles, const SkewItems& k) {
  if (item < k.base) {
    const uint32_t slice = item / splits, part = item % splits;
    if (k.heavy[slice] == k.epoch) return SliceWork{slice, slice, 0, 0};
    return SliceWork{slice, slice, n_tiles * part / splits, n_tiles * (part + 1) / splits};
  }
  const uint32_t fs = splits * k.mult, x = item - k.base, slice = x / fs, part = x % fs;
  if (k.heavy[slice] != k.epoch) return SliceWork{slice, slice, 0, 0};
  return SliceWork{slice, slice, n_tiles * part / fs, n_tiles * (part + 1) / fs};
}

// First work item >= item (stepping by gridDim.x) that has tiles; n_items if none. With skew items most of the
// fine items are empty: each lane of the wave tests one candidate (item + lane * gridDim.x) and a ballot picks
// the first with tiles, one memory round trip per 64 candidates.
__device__ __forceinline__ uint32_t next_item(uint32_t item, uint32_t n_items, uint32_t splits, uint64_t n_tiles,
                                              const uint32_t* bucket_tiles, SliceWork& sw, const SkewItems& k) {
  if (k.heavy == nullptr) {
    for (; item < n_items; item += gridDim.x) {
      sw = slice_work(xcd_item(item, n_items), splits, n_tiles, bucket_tiles);
      if (sw.t_lo < sw.t_hi) break;
    }
    return item;
  }
  const uint32_t lane = threadIdx.x & 63;
  for (; item < n_items; item += 64 * gridDim.x) {
    const uint64_t cand = static_cast<uint64_t>(item) + static_cast<uint64_t>(lane) * gridDim.x;
    SliceWork w{0, 0, 0, 0};
    if (cand < n_items) {  // each range XCD-mapped on its own: the base items land where they would without skew items
      const uint32_t c = static_cast<uint32_t>(cand);
      const uint32_t m = c < k.base ? xcd_item(c, k.base) : k.base + xcd_item(c - k.base, n_items - k.base);
      w = slice_work_skew(m, splits, n_tiles, k);
    }
    const uint64_t has = __ballot(w.t_lo < w.t_hi);
    if (has != 0) {
      const int f = __builtin_ctzll(has);
      sw.slice = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(w.slice), f));
      sw.run_row = sw.slice;
      sw.t_lo = (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(w.t_lo >> 32), f))) << 32) |
                static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(w.t_lo)), f));
      sw.t_hi = (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(w.t_hi >> 32), f))) << 32) |
                static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(w.t_hi)), f));
      return item + static_cast<uint32_t>(f) * gridDim.x;
    }
  }
  return n_items;
}

// Work items (slice, split) are walked by a resident grid; when a workgroup has several (filters with
// more slices than the chip has CUs: the bucketed strategy), the next item's slice is fetched into
// registers (128 B per thread) while the current one is probed, then stored to LDS.
__global__ __launch_bounds__(kSliceThreads) void slice_probe_kernel(const uint64_t* __restrict__ words,
                                                                   uint32_t splits, uint64_t n_tiles,
                                                                   const uint32_t* __restrict__ recs,
                                                                   const uint32_t* __restrict__ runs,
                                                                   uint8_t* __restrict__ passbits,
                                                                   uint32_t tile_cap,
                                                                   const uint32_t* __restrict__ bucket_tiles,
                                                                   uint32_t n_items, SkewItems skew) {
  // one LDS array, table first: the slice's base offset folds into the ds_read immediate
  __shared__ uint64_t s_lds[kRotMasks + kSliceWords];
  uint64_t* const s_rmasks = s_lds;
  uint64_t* const s_slice = s_lds + kRotMasks;
  u64x2* const s_slice2 = reinterpret_cast<u64x2*>(s_slice);
  __shared__ uint32_t s_win[kSliceThreads * RPT_SLICE_UNROLL];  // per-wave slot windows (16 KiB)
  constexpr uint32_t kPre = kSliceWords / 2 / kSliceThreads;  // 16-B pieces of a slice per thread
  SliceWork cur;
  uint32_t item = next_item(blockIdx.x, n_items, splits, n_tiles, bucket_tiles, cur, skew);
  if (item >= n_items) return;  // uniform
  {
    const u64x2* src = reinterpret_cast<const u64x2*>(words + static_cast<uint64_t>(cur.slice) * kSliceWords);
#pragma unroll
    for (uint32_t i = 0; i < kPre; i++) s_slice2[threadIdx.x + i * kSliceThreads] = src[threadIdx.x + i * kSliceThreads];
  }
  fill_rot_mask_table(s_rmasks);
  while (true) {
    __syncthreads();
    SliceWork nxt;
    const uint32_t nitem = next_item(item + gridDim.x, n_items, splits, n_tiles, bucket_tiles, nxt, skew);
    u64x2 pre[kPre];
    if (nitem < n_items) {
      const u64x2* src = reinterpret_cast<const u64x2*>(words + static_cast<uint64_t>(nxt.slice) * kSliceWords);
#pragma unroll
      for (uint32_t i = 0; i < kPre; i++) pre[i] = stream_load<RPT_NT_SLICE_LOADS>(src + threadIdx.x + i * kSliceThreads);
    }
    probe_slice_runs_tbl(s_slice, s_rmasks, s_win, cur, n_tiles, recs, runs, passbits, tile_cap);
    if (nitem >= n_items) break;
    __syncthreads();  // every wave is done with this slice
    for (uint32_t i = 0; i < kPre; i++) s_slice2[threadIdx.x + i * kSliceThreads] = pre[i];  // unrolled by the compiler
    item = nitem;
    cur = nxt;
  }
}

// ---- partitioned build: OR each slice's records into an LDS copy, then merge into the filter ----
// Same flattened run walk as slice_probe_kernel. Records are ORed into an LDS copy of the slice
// (ds_or_b64 per record), which is then merged into the filter by one of (`mode`):
//   kSliceMergeAtomic    LDS starts at zero; coalesced 64-bit device-scope atomic ORs of its non-zero
//                        words (several workgroups per slice compose: OR is idempotent)
//   kSliceMergeStore     the filter is all zero (rpt_bf::pristine) and this workgroup owns the slice:
//                        LDS starts at zero, the slice leaves as plain stores (all of it: whole 128-B
//                        lines; skipping the zero pieces left partial lines: 1e9 keys into a fresh
//                        8 GiB filter 10.6-11.1 ms vs 9.4 ms, tools/build_modes.py)
//   kSliceMergeAdaptive  this workgroup owns the slice: with >= kSliceWords/2 records it loads the slice
//                        into LDS first and stores it back whole (read + write at the streaming rate),
//                        with fewer it merges with atomics as above
//   kSliceMergeStoreAll  the filter's words are still to be zeroed (rpt_bf_clear is deferred) and this
//                        workgroup owns the slice: every 16-B piece is stored, zero or not, so the
//                        insert is the clear (one pass over the filter instead of a memset and a store)
// Memory-side atomics run at ~1.3 TB/s against ~6 TB/s for plain stores (MI355X_MICROARCH.md, Global
// atomics): the C5 build's merge of an 8 GiB filter took 5.8 ms with atomics. Plain writes are safe
// because the host orders every word-writing operation on a filter (rpt_bf::order_mu).
#ifndef RPT_EXP_STORE_SKIP_ZERO
#define RPT_EXP_STORE_SKIP_ZERO 0
#endif
#ifndef RPT_SLICE_INSERT_DEDUP
#define RPT_SLICE_INSERT_DEDUP 1  // drop a record equal to its slot's previous one (below)
#endif
constexpr int kSliceMergeAtomic = 0, kSliceMergeStore = 1, kSliceMergeAdaptive = 2, kSliceMergeStoreAll = 3;
__global__ __launch_bounds__(kSliceThreads) void slice_insert_kernel(uint64_t* __restrict__ words, uint32_t splits,
                                                                    uint64_t n_tiles,
                                                                    const uint32_t* __restrict__ recs,
                                                                    const uint32_t* __restrict__ runs,
                                                                    uint32_t tile_cap,
                                                                    const uint32_t* __restrict__ bucket_tiles, int mode) {
  // one LDS array, table first: the slice's base offset folds into the ds_read immediate
  __shared__ uint64_t s_lds[kRotMasks + kSliceWords];
  uint64_t* const s_rmasks = s_lds;
  uint64_t* const s_slice = s_lds + kRotMasks;
  __shared__ uint32_t s_win[kSliceThreads * RPT_SLICE_UNROLL];  // per-wave slot windows (16 KiB)
  const SliceWork sw = slice_work(xcd_item(blockIdx.x, gridDim.x), splits, n_tiles, bucket_tiles);
  const uint32_t slice = sw.slice;
  const uint64_t t_lo = sw.t_lo, t_hi = sw.t_hi;
  uint64_t* dst = words + static_cast<uint64_t>(slice) * kSliceWords;
  u64x2* const dst2 = reinterpret_cast<u64x2*>(dst);
  constexpr uint32_t kPieces = kSliceWords / 2;  // 16-B pieces of a slice
  if (t_lo >= t_hi) {  // no rows reach this slice (uniform)
    if (mode == kSliceMergeStoreAll)
      for (uint32_t i = threadIdx.x; i < kPieces; i += kSliceThreads) dst2[i] = u64x2{0, 0};
    return;
  }
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr uint32_t kWaves = kSliceThreads / 64;
  const uint32_t* my_runs = runs + static_cast<uint64_t>(sw.run_row) * n_tiles;
  u64x2* const s_slice2 = reinterpret_cast<u64x2*>(s_slice);
  bool rmw = false;
  if (mode == kSliceMergeAdaptive) {  // uniform: records this workgroup ORs into the slice
    uint32_t r = 0;
    for (uint64_t t = t_lo + threadIdx.x; t < t_hi; t += kSliceThreads) r += my_runs[t] & 0xFFFFu;
    r = wave_sum(r);
    if (lane == 0) s_win[wave] = r;
    __syncthreads();
    uint32_t tot = 0;
    for (uint32_t w = 0; w < kWaves; w++) tot += s_win[w];
    rmw = tot >= kSliceWords / 2;
    __syncthreads();
  }
  if (rmw) {
    for (uint32_t i = threadIdx.x; i < kPieces; i += kSliceThreads) s_slice2[i] = dst2[i];
  } else {
    for (uint32_t i = threadIdx.x; i < kSliceWords; i += kSliceThreads) s_slice[i] = 0;
  }
  fill_rot_mask_table(s_rmasks);
  __syncthreads();
  const uint32_t bt = batch_tiles(t_hi - t_lo);  // as slice_probe_kernel
  // slot -> run through the wave's LDS window, as probe_slice_runs_tbl
  constexpr uint32_t kWin = 64 * RPT_SLICE_UNROLL;
  uint32_t* win = s_win + wave * kWin;
  for (uint64_t tb = t_lo + wave * bt; tb < t_hi; tb += kWaves * bt) {
    const uint32_t info = (lane < bt && tb + lane < t_hi) ? my_runs[tb + lane] : 0u;
    const uint32_t real = info & 0xFFFFu;  // records of the run (pad slots are stale)
    const uint32_t nslot = pad_run(real) / kRunPad;
    const uint32_t base = (lane * tile_cap + (info >> 16)) / kRunPad;  // first slot, relative to the batch
    const uint32_t* brecs = recs + tb * tile_cap;                     // uniform
    const uint32_t incl = wave_inclusive_sum(nslot);
    const uint32_t excl = incl - nslot;
    const uint32_t total = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), 63));
    const int base_m_excl = static_cast<int>(base - excl);
    const int real_p_excl = static_cast<int>(real + excl * kRunPad);  // real records before slot s: s*8 - excl*8
    for (uint32_t w0 = 0; w0 < total; w0 += kWin) {
#pragma unroll
      for (int u = 0; u < RPT_SLICE_UNROLL; u++) win[u * 64 + lane] = 0u;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (nslot != 0 && excl < w0 + kWin && incl > w0) win[(excl > w0 ? excl : w0) - w0] = lane + 1;
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
      uint32_t nreal[RPT_SLICE_UNROLL];
      u32x4 rec[RPT_SLICE_UNROLL][2];
      uint32_t carry = 0;
#pragma unroll
      for (int u = 0; u < RPT_SLICE_UNROLL; u++) {
        const uint32_t slot = w0 + u * 64 + lane;
        uint32_t m = wave_inclusive_max(win[u * 64 + lane]);
        m = max(m, carry);
        carry = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(m), 63));
        const int src = static_cast<int>(m - 1) << 2;
        const uint32_t rel = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, base_m_excl)) + slot;
        const int left = __builtin_amdgcn_ds_bpermute(src, real_p_excl) - static_cast<int>(slot * kRunPad);
        nreal[u] = (slot < total && left > 0) ? (left < static_cast<int>(kRunPad) ? static_cast<uint32_t>(left) : kRunPad) : 0u;
        rec[u][0] = rec[u][1] = u32x4{0, 0, 0, 0};
        if (w0 + u * 64 < total && nreal[u] != 0) {
          rec[u][0] = *reinterpret_cast<const u32x4*>(brecs + rel * kRunPad);
          rec[u][1] = *reinterpret_cast<const u32x4*>(brecs + rel * kRunPad + 4);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int u = 0; u < RPT_SLICE_UNROLL; u++) {
        if (w0 + u * 64 >= total) break;  // uniform
        // a record equal to the slot's previous one (same word, same mask) ORs nothing new: LDS atomics on one
        // word serialize (one key repeated 4 Mi times: 3.7 ms, profiles/r05/insert_duplicates.jsonl)
#pragma unroll
        for (uint32_t e = 0; e < kRunPad; e++) {
          if (e < nreal[u] && (!RPT_SLICE_INSERT_DEDUP || e == 0 || rec[u][e >> 2][e & 3] != rec[u][(e - 1) >> 2][(e - 1) & 3])) {
            const uint32_t rec1 = rec[u][e >> 2][e & 3];
            atomicOr(reinterpret_cast<unsigned long long*>(&s_slice[rec_word(rec1)]),
                     static_cast<unsigned long long>(rec_mask(s_rmasks, rec1)));
          }
        }
      }
    }
  }
  __syncthreads();
  if (rmw) {
    for (uint32_t i = threadIdx.x; i < kPieces; i += kSliceThreads) dst2[i] = s_slice2[i];
  } else if (mode == kSliceMergeStore || mode == kSliceMergeStoreAll) {
    for (uint32_t i = threadIdx.x; i < kPieces; i += kSliceThreads) {
      const u64x2 v = s_slice2[i];
      if (RPT_EXP_STORE_SKIP_ZERO && mode == kSliceMergeStore && (v[0] | v[1]) == 0) continue;  // A/B only
      dst2[i] = v;
    }
  } else {
    for (uint32_t i = threadIdx.x; i < kSliceWords; i += kSliceThreads) {
      const uint64_t v = s_slice[i];
      if (v) __hip_atomic_fetch_or(dst + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// The pass bits of the two rows whose u16 record positions share the 32-bit row-map word w (bit 0: the
// low half's row). The unpermute kernels run close to VALU-bound (C2 unpermute_sel: 0.81 VALU instructions
// per CU cycle), so: the bits are read as 32-bit LDS words from a STATIC array (its base folds into the
// instruction's offset; a dynamic array's base is a link-time symbol the compiler adds per lookup), and
// v_bfe_u32 takes the bit offset from the low 5 bits of its operand, so the low position needs no mask.
template <int TM>
constexpr uint32_t kPassWordsMax = static_cast<uint32_t>(tile_cap_for(kMaxSliceCount, TM) / 32);
__device__ __forceinline__ uint32_t pass_bits2(const uint32_t* s_pass32, uint32_t w) {
  const uint32_t hi = w >> 16;
  return __builtin_amdgcn_ubfe(s_pass32[(w & 0xFFFFu) >> 5], w, 1) | (__builtin_amdgcn_ubfe(s_pass32[hi >> 5], hi, 1) << 1);
}
// ---- partitioned probe, C: restore row order -> result bits + per-segment counts (P1's format) -----
// One 256-thread workgroup per tile: the tile's pass bits (tile_cap / 8 bytes) are staged in LDS while
// each wave's row positions are already in flight; a lane owns 8 consecutive rows of a segment (one
// 16-B load of positions) and produces byte `lane` of the segment's 512-bit row-ordered result.
constexpr int kUnpermuteThreads = 256;
template <int TM>
__global__ __launch_bounds__(kUnpermuteThreads) void unpermute_kernel(const uint16_t* __restrict__ pos,
                                                                     const uint8_t* __restrict__ passbits, uint64_t n,
                                                                     uint64_t tile_cap,
                                                                     uint64_t* __restrict__ out_bits,
                                                                     uint32_t* __restrict__ seg_counts,
                                                                     const uint32_t* __restrict__ dev_n_tiles) {
  if (dev_n_tiles != nullptr && blockIdx.x >= *dev_n_tiles) return;  // bucketed: grid is an upper bound
  __shared__ uint32_t s_pass[kPassWordsMax<TM>];  // tile_cap / 8 bytes of pass bits (record order)
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t n_segs = (n + kSegRows - 1) / kSegRows;
  constexpr uint32_t kSegsPerWave = (kTileRows * TM / kSegRows) / (kUnpermuteThreads / 64);
  const uint64_t tile = blockIdx.x;
  const uint64_t seg0 = tile * (kTileRows * TM / kSegRows) + wave * kSegsPerWave;
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
    for (int c = 0; c < 4; c++) byte |= pass_bits2(s_pass, pv[sg][c]) << (2 * c);
    const uint64_t row0 = seg * kSegRows + lane * 8;  // rows >= n (last segment) carry don't-care positions
    if (row0 + 8 > n) byte = row0 >= n ? 0u : byte & ((1u << (n - row0)) - 1u);
    out_bytes[seg * (kSegRows / 8) + lane] = static_cast<uint8_t>(byte);
    if (seg_counts != nullptr) {
      const uint32_t cnt = wave_sum(__popc(byte));
      if (lane == 0) seg_counts[seg] = cnt;
    }
  }
}
}  // namespace rpt

namespace rpt {
// ---- partitioned probe, C': restore row order straight into the selection vector -----------------
// LookupSel's fused tail (rpt_bf_probe, PARTITIONED strategy): a tile's survivor count is the
// popcount of its pass bits (the slice probe writes 0 for pad slots), so the tiles' output offsets are
// known before the unpermute. The unpermute then writes ascending row ids directly. This replaces
// the result bit vector, its per-segment counts, and the separate compaction pass.

// C'1: survivors per tile: popcount of the tile's used pass-bit bytes (its padded runs), one wave per tile.
constexpr int kTileCountThreads = 256;
__global__ __launch_bounds__(kTileCountThreads) void tile_count_kernel(const uint8_t* __restrict__ passbits,
                                                                      const uint32_t* __restrict__ runs_tm,
                                                                      uint32_t n_slices, uint64_t n_tiles,
                                                                      uint64_t tile_cap,
                                                                      uint32_t* __restrict__ tile_counts) {
  const uint64_t tile = static_cast<uint64_t>(blockIdx.x) * (kTileCountThreads / 64) + (threadIdx.x >> 6);
  if (tile >= n_tiles) return;  // wave-uniform
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t last = runs_tm[tile * n_slices + n_slices - 1];  // the last slice's run ends the used records
  const uint32_t used = ((last >> 16) + pad_run(last & 0xFFFFu)) / kRunPad;  // bytes of pass bits
  const u32x4* blk = reinterpret_cast<const u32x4*>(passbits + tile * (tile_cap / kRunPad));
  uint32_t c = 0;
  for (uint32_t i = lane; i * 16 < used; i += 64) {
    const u32x4 v = blk[i];
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const uint32_t b0 = i * 16 + e * 4;  // first byte of this word
      uint32_t w = v[e];
      if (b0 + 4 > used) w = b0 >= used ? 0u : w & ((1u << (8 * (used - b0))) - 1u);
      c += __popc(w);
    }
  }
  c = wave_sum(c);
  if (lane == 0) tile_counts[tile] = c;
}

// C'1b: blocks of 256 tiles: each tile's exclusive prefix inside its block (in place) + the block sums
// (group_scan_kernel then scans the few block sums).
constexpr int kTileBlock = 256;
__global__ __launch_bounds__(kTileBlock) void tile_block_scan_kernel(uint32_t* __restrict__ tile_counts, uint64_t n_tiles,
                                                                    uint32_t* __restrict__ block_sums) {
  __shared__ uint32_t s_w[kTileBlock / 64];
  const uint64_t t = static_cast<uint64_t>(blockIdx.x) * kTileBlock + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t c = t < n_tiles ? tile_counts[t] : 0u;
  const uint32_t inc = wave_inclusive_sum(c);
  if (lane == 63) s_w[wave] = inc;
  __syncthreads();
  uint32_t off = 0, all = 0;
  for (uint32_t w = 0; w < kTileBlock / 64; w++) {
    off += w < wave ? s_w[w] : 0u;
    all += s_w[w];
  }
  if (t < n_tiles) tile_counts[t] = off + inc - c;
  if (threadIdx.x == 0) block_sums[blockIdx.x] = all;
}

// C'2 (tile_pre = prefix inside the tile's block, block_offs = the blocks' scan). 256 threads per 16 Ki
// rows (8 segments per wave at either tile size: 32 Ki-row tiles get 512 threads, not 16 segments'
// worth of row-map registers per lane).: one 256-thread workgroup per
// tile, as unpermute_kernel; each wave's segments are consecutive rows, so a survivor's sel index is
// tile offset + earlier waves' survivors + earlier segments of this wave + earlier lanes of its segment.
template <int TM>
constexpr int kUnpermuteSelThreads = kUnpermuteThreads * TM;
template <int TM>
__global__ __launch_bounds__(kUnpermuteSelThreads<TM>) void unpermute_sel_kernel(const uint16_t* __restrict__ pos,
                                                                         const uint8_t* __restrict__ passbits,
                                                                         uint64_t n, uint64_t tile_cap,
                                                                         const uint32_t* __restrict__ tile_pre,
                                                                         const uint32_t* __restrict__ block_offs,
                                                                         const uint32_t* __restrict__ row_sel,
                                                                         uint32_t* __restrict__ out_sel) {
  __shared__ uint32_t s_pass[kPassWordsMax<TM>];  // tile_cap / 8 bytes of pass bits (record order)
  constexpr int kThreads = kUnpermuteSelThreads<TM>;
  __shared__ uint32_t s_wtot[kThreads / 64];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t n_segs = (n + kSegRows - 1) / kSegRows;
  constexpr uint32_t kSegsPerWave = (kTileRows * TM / kSegRows) / (kThreads / 64);
  const uint64_t tile = blockIdx.x;
  const uint64_t seg0 = tile * (kTileRows * TM / kSegRows) + wave * kSegsPerWave;
  u32x4 pv[kSegsPerWave];  // 8 row positions (u16) per lane per segment
#pragma unroll
  for (uint32_t sg = 0; sg < kSegsPerWave; sg++) {
    pv[sg] = u32x4{0, 0, 0, 0};
    if (seg0 + sg < n_segs)
      pv[sg] = stream_load<RPT_NT_REC_LOADS>(reinterpret_cast<const u32x4*>(pos + (seg0 + sg) * kSegRows + lane * 8));
  }
  {
    const u32x4* src = reinterpret_cast<const u32x4*>(passbits + tile * (tile_cap / 8));
    for (uint32_t i = threadIdx.x; i < tile_cap / 128; i += kThreads) reinterpret_cast<u32x4*>(s_pass)[i] = src[i];
  }
  __syncthreads();
  uint32_t bytes[kSegsPerWave], excl[kSegsPerWave], segtot[kSegsPerWave], run = 0;
#pragma unroll
  for (uint32_t sg = 0; sg < kSegsPerWave; sg++) {
    uint32_t byte = 0;
#pragma unroll
    for (int c = 0; c < 4; c++) byte |= pass_bits2(s_pass, pv[sg][c]) << (2 * c);
    const uint64_t row0 = (seg0 + sg) * kSegRows + lane * 8;  // rows >= n carry don't-care positions
    if (row0 + 8 > n) byte = row0 >= n ? 0u : byte & ((1u << (n - row0)) - 1u);
    bytes[sg] = byte;
    const uint32_t c = __popc(byte);
    const uint32_t inc = wave_inclusive_sum(c);
    excl[sg] = run + inc - c;
    segtot[sg] = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(inc), 63));
    run += segtot[sg];
  }
  if (lane == 0) s_wtot[wave] = run;
  __syncthreads();
  uint32_t woff = block_offs[tile / kTileBlock] + tile_pre[tile];
  for (uint32_t w = 0; w < wave; w++) woff += s_wtot[w];
#if RPT_SEL_BALLOT_EXPAND
  // Dense segments (>= RPT_SEL_BALLOT_MIN survivors of 512): row-ordered 64-row words (lane 8k + j holds
  // byte j of word k; the bytes are ORed within each group of 8 lanes by DPP), expanded word by word
  // so each store writes one contiguous run of survivors. Sparse segments: each lane writes its own
  // survivors (fewer instructions when a lane has ~1). Measured (C2 unpermute_sel ms, p = 0.1 / 0.5 /
  // 1.0): per-lane only 0.48 / 1.09 / 2.89, word-by-word only 0.65 / 0.80 / 1.15; C2 step at p = 0.25
  // with the switch at 64 / 128 / 192 survivors: 4.12 / 4.10 / 4.08 ms (per-lane only 4.08).
  uint32_t o = woff;
#pragma unroll
  for (uint32_t sg = 0; sg < kSegsPerWave; sg++) {
    if (segtot[sg] < RPT_SEL_BALLOT_MIN) {  // uniform
      uint32_t b = bytes[sg], ol = woff + excl[sg];
      const uint32_t row0 = static_cast<uint32_t>((seg0 + sg) * kSegRows) + lane * 8;
      while (b) {
        const uint32_t row = row0 + static_cast<uint32_t>(__builtin_ctz(b));
        out_sel[ol++] = row_sel ? row_sel[row] : row;
        b &= b - 1;
      }
      o += segtot[sg];
      continue;
    }
    uint64_t v = static_cast<uint64_t>(bytes[sg]) << (8 * (lane & 7));
    uint32_t lo = static_cast<uint32_t>(v), hi = static_cast<uint32_t>(v >> 32);
    lo |= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(lo), 0xB1, 0xf, 0xf, false));
    hi |= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(hi), 0xB1, 0xf, 0xf, false));
    lo |= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(lo), 0x4E, 0xf, 0xf, false));
    hi |= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(hi), 0x4E, 0xf, 0xf, false));
    lo |= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(lo), 0x141, 0xf, 0xf, false));
    hi |= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(hi), 0x141, 0xf, 0xf, false));
    v = (static_cast<uint64_t>(hi) << 32) | lo;
    const uint32_t row0 = static_cast<uint32_t>((seg0 + sg) * kSegRows);
#pragma unroll
    for (int k = 0; k < 8; k++) o += expand_word_sel(readlane64(v, 8 * k), row0 + 64 * k, lane, row_sel, out_sel + o);
  }
#else
#pragma unroll
  for (uint32_t sg = 0; sg < kSegsPerWave; sg++) {
    uint32_t b = bytes[sg], o = woff + excl[sg];
    const uint32_t row0 = static_cast<uint32_t>((seg0 + sg) * kSegRows) + lane * 8;
    while (b) {
      const uint32_t row = row0 + static_cast<uint32_t>(__builtin_ctz(b));
      out_sel[o++] = row_sel ? row_sel[row] : row;
      b &= b - 1;
    }
  }
#endif
}
}  // namespace rpt
