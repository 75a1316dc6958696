// bucketed.hpp — level 1 of the bucketed (two-level) strategy for filters of 32 MiB..16 GiB.
// Part of librpt_gpu.so: included by rpt_gpu.hip (one translation unit: kernels and their launches
// stay together without relocatable device code).
#pragma once

namespace rpt {

// ---- bucketed strategy (filters of 2^22..2^31 blocks) ----------------------------------------------
// Level 1 cuts the rows by 32 MiB filter region ("bucket": 256 slices) in ONE pass over the keys; level 2
// is the partitioned pipeline over the resulting level-2 hash array, every bucket against its own 256
// slices. bucket = block id >> 22 = hash bits 38...
//
// The level-2 array is built without a counting pass (r02 read the keys twice: a count kernel for the
// bucket totals, then the scatter). Each level-1 tile (16 Ki rows) sorts its rows by bucket in LDS and
// APPENDS each bucket's run to a list: list (g, b) for bucket b and group g = the workgroup's XCD (8
// groups, so a list's neighbouring runs leave one L2 and merge there into whole lines; 1 group for
// small batches, where 8 lists per bucket would pad too much). A list is a sequence of 4 Ki-row chunks: a
// run's rows [p, p + c) of its list come from one returning atomic on the list's row cursor, whose
// latency overlaps the LDS sort. The first K chunks of every list have fixed ids (list * K + c; K = 1 by
// default, rpt_gpu.hip RPT_L1_FIXED_PCT). Beyond K a list grows by extents of kExtentChunks chunks
// taken from its group's pool shard (one atomic per 64 Ki rows of a list): the run that
// covers an extent's first row takes it and publishes its first chunk id in ext_dir; a run that starts
// inside an extent someone else took waits for that id (its taker did its cursor atomic earlier and
// publishes before waiting for anything, so it finishes; the wait is bounded anyway and flags `error`).
// bucket_lists_kernel then lays every bucket's lists out as consecutive level-2 tiles of 4 chunks
// ("w-space": the row order level 2 sees) through chunk_map, and pads each list's last chunk with copies
// of one of its hashes (re-inserting or re-probing a present hash changes nothing; the pads' results are
// never read).
static_assert(kLogNumMasks + 6 + kSliceLog + kBucketSliceLog <= 40, "level-2 split hashes carry bits 0..39");
__device__ __forceinline__ uint32_t bucket_of(uint64_t h, uint32_t bucket_mask) {
  return static_cast<uint32_t>(h >> (kLogNumMasks + 6 + kSliceLog + kBucketSliceLog)) & bucket_mask;
}

constexpr uint32_t kChunkEmpty = ~0u;        // an extent not taken yet
constexpr uint32_t kChunkInvalid = ~0u - 1;  // beyond the list's extent bound (never expected: flags `error`)
constexpr uint32_t kMaxRunChunks = static_cast<uint32_t>(kL1TileRows / kChunkRows) + 1;  // chunks one run can touch
constexpr uint32_t kL1Groups = 8;
constexpr uint32_t kExtentChunks = 16;          // overflow extents: 64 Ki rows
constexpr uint32_t kChunkSpinLimit = 1u << 22;  // ~0.3 s of polling: never reached unless a kernel is broken

struct L1Lists {
  uint32_t* cursor;     // [groups * nb] rows appended to each list        } zeroed before the scatter
  uint32_t* pool;       // [groups] extents taken from each group's shard   }
  uint32_t* error;      // [1] a bound was hit (never expected)             }
  uint32_t* ext_dir;    // [groups * nb][n_ext] first chunk id of a list's e-th extent (kChunkEmpty until taken)
  uint32_t k_fixed;     // K: chunks with fixed ids per list
  uint32_t n_ext;       // extents per list (bound)
  uint32_t shard_ext;   // extents per pool shard (bound)
  uint32_t groups;      // 1 or kL1Groups
  uint32_t n_lists;     // groups * nb
};

// Chunk id of chunk c of list `list` when it is a fixed one or its extent is published (else kChunkEmpty,
// or kChunkInvalid past the list's extent bound).
__device__ __forceinline__ uint32_t l1_chunk_id(const L1Lists& L, uint64_t list, uint32_t c) {
  if (c < L.k_fixed) return static_cast<uint32_t>(list * L.k_fixed + c);
  const uint32_t x = c - L.k_fixed, e = x / kExtentChunks;
  if (e >= L.n_ext) return kChunkInvalid;
  const uint32_t base = __hip_atomic_load(&L.ext_dir[list * L.n_ext + e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return base == kChunkEmpty ? kChunkEmpty : base + x % kExtentChunks;
}

// Level-1 tiles are mapped XCD-contiguously (workgroup b runs on XCD b % 8): each XCD gets a contiguous
// tile range. The list group of a tile is the XCD share of the workgroup that scattered it.
__device__ __forceinline__ uint64_t l1_tile_of_block(uint32_t blk, uint32_t grid) {
  const uint32_t per = grid / kL1Groups;
  return blk < per * kL1Groups ? static_cast<uint64_t>(blk % kL1Groups) * per + blk / kL1Groups : blk;
}
__device__ __forceinline__ uint32_t l1_group_of_tile(uint64_t tile, uint32_t grid, uint32_t groups) {
  if (groups == 1) return 0;
  const uint32_t per = grid / kL1Groups;
  return tile < static_cast<uint64_t>(per) * kL1Groups ? static_cast<uint32_t>(tile / per)
                                                      : static_cast<uint32_t>(tile % kL1Groups);
}

__device__ __forceinline__ void l1_flag_error(const L1Lists& L) {
  __hip_atomic_store(L.error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The scatter's row map (pos_out) leaves as one 2V-byte store per lane for dense keys (1), non-temporal like
// the partition's (2), or as V strided u16 stores (0): scatter 2.967-3.006 -> 2.940-2.969 ms with 2, C5 share
// 8.47-8.52 -> 8.44-8.47 ms (profiles/r04/ab_scatter_pos_pack.txt).
#ifndef RPT_SCATTER_POS_PACK
#define RPT_SCATTER_POS_PACK 2
#endif
// B1: one pass over a 16 Ki-row level-1 tile: hash every row (held in registers), rank it within its
// bucket (LDS atomic), append each bucket's run to its list (see above), sort the tile's hashes by
// bucket in LDS and copy them to their list positions as the level-2 kKeySplit layout: hash bits 0..31
// in hash_lo, bits 32..39 in hash_hi. Probe only: pos_out (u16) = each row's slot in the tile's
// bucket-sorted order, counts_tm / pre_tm [tile][bucket] = the run's length and its start in its list.
// Build only (MM): the key min/max is folded into stats.
template <int K, bool DENSE, bool MM>
__global__ __launch_bounds__(kTileThreads) void bucket_scatter_kernel(KeyArgs a, uint64_t n, uint32_t bucket_mask, L1Lists L,
                                                                      uint32_t* __restrict__ hash_lo,
                                                                      uint8_t* __restrict__ hash_hi,
                                                                      uint16_t* __restrict__ pos_out,
                                                                      uint32_t* __restrict__ counts_tm,
                                                                      uint32_t* __restrict__ pre_tm,
                                                                      int64_t* __restrict__ stats) {
  extern __shared__ uint64_t s_h[];  // kL1TileRows hashes, bucket-sorted (one 8-B LDS write per row; the
                                     // bucket, bits 38.., is re-derived on the way out)
  __shared__ uint32_t s_cnt[kMaxBuckets], s_start[kMaxBuckets];
  __shared__ uint64_t s_qc[kMaxBuckets];  // (list position of sorted slot 0) | first chunk index << 32
  __shared__ uint32_t s_chunk[kMaxRunChunks][kMaxBuckets];  // ids of the chunks the run covers
  __shared__ int64_t s_mm[kTileThreads / 64][2];             // MM: each wave's key min / max
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t nb = bucket_mask + 1;
  const uint64_t tile = l1_tile_of_block(blockIdx.x, gridDim.x);
  const uint32_t grp = L.groups == 1 ? 0u : blockIdx.x % kL1Groups;
  const uint64_t tile_base = tile * kL1TileRows;
  // the threads that own a bucket's list (the last kMaxBuckets threads: wave 0 scans meanwhile)
  const uint32_t own_b = threadIdx.x - (kTileThreads - kMaxBuckets);
  const bool owner = threadIdx.x >= kTileThreads - kMaxBuckets && own_b < nb;
  for (uint32_t i = threadIdx.x; i < nb; i += kTileThreads) s_cnt[i] = 0;
  // MM: the filter's min / max as of now, loaded early and compared at the end (they only ever improve, so
  // a workgroup whose keys cannot improve the early values cannot improve the current ones either)
  [[maybe_unused]] int64_t pre_mn = kMinInit, pre_mx = kMaxInit;
  if constexpr (MM && KeyTraits<K>::kValues) {
    if (threadIdx.x == 0) {
      pre_mn = __hip_atomic_load(stats, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      pre_mx = __hip_atomic_load(stats + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  uint64_t hh[kL1SegsPerWave][8];
  uint32_t rk[kL1SegsPerWave][8];  // rank within the bucket, ~0 for rows past n
  int64_t mm[2] = {kMinInit, kMaxInit};  // MM: this lane's key min / max over the tile
#pragma unroll
  for (int sg = 0; sg < kL1SegsPerWave; sg++) {
    const uint64_t sbase = tile_base + wave * (kL1SegsPerWave * kSegRows) + sg * kSegRows;
    bool oo[8];
    load_hashes<K, DENSE, MM, false, true>(a, sbase, n, lane, hh[sg], oo, mm);
#pragma unroll
    for (int j = 0; j < 8; j++) rk[sg][j] = oo[j] ? atomicAdd(&s_cnt[bucket_of(hh[sg][j], bucket_mask)], 1u) : ~0u;
  }
  if constexpr (MM && KeyTraits<K>::kValues) {
    wave_minmax(mm[0], mm[1]);
    if (lane == 0) {
      s_mm[wave][0] = mm[0];
      s_mm[wave][1] = mm[1];
    }
  }
  __syncthreads();
  uint32_t run_p = 0, run_c = 0;  // owner: the run's start in its list and its length
  const uint64_t list = static_cast<uint64_t>(grp) * nb + own_b;
  if (wave == 0) {  // exclusive scan of the bucket counts, kMaxBuckets / 64 per lane
    constexpr int kPer = kMaxBuckets / 64;
    uint32_t c[kPer], t = 0;
#pragma unroll
    for (int i = 0; i < kPer; i++) {
      const uint32_t idx = lane * kPer + i;
      c[i] = idx < nb ? s_cnt[idx] : 0u;
      t += c[i];
    }
    uint32_t off = wave_inclusive_sum(t) - t;
#pragma unroll
    for (int i = 0; i < kPer; i++) {
      const uint32_t idx = lane * kPer + i;
      if (idx < nb) s_start[idx] = off;
      off += c[i];
    }
  } else if (owner) {  // append the run to its list (the returned start is used after the LDS sort)
    run_c = s_cnt[own_b];
    if (run_c != 0) run_p = atomicAdd(&L.cursor[list], run_c);
  }
  __syncthreads();
  // the rows to their bucket-sorted LDS slots; the row map gets the slot
#pragma unroll
  for (int sg = 0; sg < kL1SegsPerWave; sg++) {
    const uint64_t sbase = tile_base + wave * (kL1SegsPerWave * kSegRows) + sg * kSegRows;
    uint16_t pv[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint32_t p = 0;
      if (rk[sg][j] != ~0u) {
        const uint32_t b = bucket_of(hh[sg][j], bucket_mask);
        p = s_start[b] + rk[sg][j];
        s_h[p] = hh[sg][j];
      }
      pv[j] = static_cast<uint16_t>(p);
    }
    if (pos_out == nullptr) {  // padded to whole tiles: rows >= n get don't-care values
    } else if constexpr (DENSE && RPT_SCATTER_POS_PACK) {
      // a lane's V adjacent rows leave as one 2V-byte store (one coalesced 128 / 256-B piece per
      // instruction instead of V strided u16 stores that each half-fill their lines)
      constexpr int V = KeyTraits<K>::kVec;
#pragma unroll
      for (int c = 0; c < 8 / V; c++) {
        const uint64_t row0 = sbase + static_cast<uint64_t>(c) * 64 * V + static_cast<uint64_t>(lane) * V;
        if constexpr (V == 2) {
          part_store<RPT_SCATTER_POS_PACK == 2>(reinterpret_cast<uint32_t*>(pos_out + row0),
                                                static_cast<uint32_t>(pv[c * 2]) | (static_cast<uint32_t>(pv[c * 2 + 1]) << 16));
        } else {
          part_store<RPT_SCATTER_POS_PACK == 2>(reinterpret_cast<uint64_t*>(pos_out + row0),
                                                static_cast<uint64_t>(pv[c * 4]) | (static_cast<uint64_t>(pv[c * 4 + 1]) << 16) |
                                                    (static_cast<uint64_t>(pv[c * 4 + 2]) << 32) |
                                                    (static_cast<uint64_t>(pv[c * 4 + 3]) << 48));
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; j++) pos_out[sbase + seg_row<K, DENSE>(j, lane)] = pv[j];
    }
  }
  if (owner) {
    if (counts_tm != nullptr) {
      counts_tm[tile * nb + own_b] = run_c;
      pre_tm[tile * nb + own_b] = run_p;
    }
    if (run_c != 0) {
      const uint32_t c0 = run_p >> kChunkLog, c1 = (run_p + run_c - 1) >> kChunkLog;
      if (c1 >= L.k_fixed) {
        // take the extents whose first row this run covers (publishing before any wait) ...
        for (uint32_t cc = max(c0, L.k_fixed); cc <= c1; cc++) {
          const uint32_t x = cc - L.k_fixed;
          if (x % kExtentChunks != 0 || (static_cast<uint64_t>(cc) << kChunkLog) < run_p) continue;
          const uint32_t e = x / kExtentChunks, local = atomicAdd(&L.pool[grp], 1u);
          if (e >= L.n_ext || local >= L.shard_ext) {
            l1_flag_error(L);
            continue;
          }
          const uint32_t first = L.n_lists * L.k_fixed + (grp * L.shard_ext + local) * kExtentChunks;
          __hip_atomic_store(&L.ext_dir[list * L.n_ext + e], first, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      // ... then the ids of the chunks the run covers (fixed, own extents, or an extent an earlier run took)
      for (uint32_t cc = c0; cc <= c1; cc++) {
        uint32_t id, spins = 0;
        for (;;) {
          id = l1_chunk_id(L, list, cc);
          if (id == kChunkInvalid || (id == kChunkEmpty && ++spins > kChunkSpinLimit)) {
            l1_flag_error(L);  // copy the run into chunk 0 (in bounds); the result degrades, see B2 / B6
            id = 0;
            break;
          }
          if (id != kChunkEmpty) break;
          __builtin_amdgcn_s_sleep(2);
        }
        s_chunk[cc - c0][own_b] = id;
      }
      s_qc[own_b] = static_cast<uint64_t>(run_p - s_start[own_b]) | (static_cast<uint64_t>(c0) << 32);
    }
  }
  __syncthreads();
  // copy-out over the tile's bucket-sorted rows, every lane busy: a wave's 64 rows span ~2 runs, so each
  // store instruction writes whole pieces of runs
  const uint32_t used = s_start[nb - 1] + s_cnt[nb - 1];
  for (uint32_t i = threadIdx.x; i < used; i += kTileThreads) {
    const uint64_t h = s_h[i];
    const uint32_t b = bucket_of(h, bucket_mask);
    const uint64_t qc = s_qc[b];
    const uint32_t q = static_cast<uint32_t>(qc) + i;  // the row's position in its list
    const uint32_t k = (q >> kChunkLog) - static_cast<uint32_t>(qc >> 32);
    const uint64_t d = static_cast<uint64_t>(s_chunk[k][b]) * kChunkRows + (q & (kChunkRows - 1));
#ifndef RPT_EXP_SCATTER_SKIP
#define RPT_EXP_SCATTER_SKIP 0  // measurement only: 1 = no high-byte stores, 2 = no low-word stores, 3 = neither
#endif
    if (!(RPT_EXP_SCATTER_SKIP & 2)) hash_lo[d] = static_cast<uint32_t>(h);
    if (!(RPT_EXP_SCATTER_SKIP & 1)) hash_hi[d] = static_cast<uint8_t>(h >> 32);
  }
  if constexpr (MM && KeyTraits<K>::kValues) {
    if (threadIdx.x == 0) {  // one publish per workgroup; no-return atomics, nothing waits on them
      int64_t mn = kMinInit, mx = kMaxInit;
      for (int w = 0; w < kTileThreads / 64; w++) {
        mn = min(mn, s_mm[w][0]);
        mx = max(mx, s_mm[w][1]);
      }
      if (mn < pre_mn) (void)__hip_atomic_fetch_min(stats, mn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (mx > pre_mx) (void)__hip_atomic_fetch_max(stats + 1, mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// B2: per bucket (one workgroup each): its level-2 tiles are its lists' chunks in group order, 4 per tile,
// the last tile completed with copies of the bucket's last chunk (rows past the lists' ends are never
// read back); list_base[g][b] = the w-space row of list (g, b)'s first row; bucket_tiles[b] = the
// bucket's first tile, bucket_tiles[nb] = the tile count (0 if the scatter flagged an error: level 2 then
// runs on nothing, and the result degrades to the conservative one, never to a false negative: a probe
// passes every row (B6), an insert sets every filter bit (l1_error_fill_kernel)). Each list's last chunk is
// padded with copies of its first row.
constexpr int kListsThreads = 256;
__global__ __launch_bounds__(kListsThreads) void bucket_lists_kernel(L1Lists L, uint32_t nb, uint32_t* __restrict__ chunk_map,
                                                                    uint64_t* __restrict__ list_base,
                                                                    uint32_t* __restrict__ bucket_tiles,
                                                                    uint32_t* __restrict__ hash_lo,
                                                                    uint8_t* __restrict__ hash_hi) {
  __shared__ uint32_t s_red[kListsThreads / 64];
  __shared__ uint32_t s_k[kL1Groups + 1];  // prefix over the bucket's lists of their chunk counts
  const uint32_t b = blockIdx.x, G = L.groups;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t acc = 0;  // tiles of the buckets before b
  for (uint32_t bb = threadIdx.x; bb < b; bb += kListsThreads) {
    uint32_t kk = 0;
    for (uint32_t g = 0; g < G; g++) kk += static_cast<uint32_t>((L.cursor[g * nb + bb] + kChunkRows - 1) >> kChunkLog);
    acc += (kk + kChunksPerTile - 1) / kChunksPerTile;
  }
  acc = wave_sum(acc);
  if (lane == 0) s_red[wave] = acc;
  if (threadIdx.x == 0) {
    uint32_t kk = 0;
    for (uint32_t g = 0; g < G; g++) {
      s_k[g] = kk;
      kk += static_cast<uint32_t>((L.cursor[g * nb + b] + kChunkRows - 1) >> kChunkLog);
    }
    s_k[G] = kk;
  }
  __syncthreads();
  uint32_t first = 0;
  for (uint32_t w = 0; w < kListsThreads / 64; w++) first += s_red[w];
  const uint32_t nk = s_k[G], tiles = (nk + kChunksPerTile - 1) / kChunksPerTile;
  const bool err = *L.error != 0;
  if (threadIdx.x < G) list_base[threadIdx.x * nb + b] = (static_cast<uint64_t>(first) * kChunksPerTile + s_k[threadIdx.x]) * kChunkRows;
  if (threadIdx.x == 0) {
    bucket_tiles[b] = err ? 0u : first;
    if (b == nb - 1) bucket_tiles[nb] = err ? 0u : first + tiles;
  }
  for (uint32_t j = threadIdx.x; j < tiles * kChunksPerTile; j += kListsThreads) {
    const uint32_t jj = min(j, nk - 1);
    uint32_t g = 0;
    while (g + 1 < G && s_k[g + 1] <= jj) g++;
    chunk_map[static_cast<uint64_t>(first) * kChunksPerTile + j] = l1_chunk_id(L, static_cast<uint64_t>(g) * nb + b, jj - s_k[g]);
  }
  if (err) return;
  for (uint32_t g = 0; g < G; g++) {
    const uint32_t rows = L.cursor[g * nb + b], r = rows & (kChunkRows - 1);
    if (r == 0) continue;  // uniform
    const uint64_t c0 = static_cast<uint64_t>(l1_chunk_id(L, static_cast<uint64_t>(g) * nb + b, rows >> kChunkLog)) * kChunkRows;
    const uint32_t lo = hash_lo[c0];
    const uint8_t hi = hash_hi[c0];
    for (uint32_t i = r + threadIdx.x; i < kChunkRows; i += kListsThreads) {
      hash_lo[c0 + i] = lo;
      hash_hi[c0 + i] = hi;
    }
  }
}

// B6: level-1 unpermute. Per level-1 tile: gather the pass bits of its bucket runs out of the level-2
// result bits (bits2, level-2 array order) into LDS in the tile's bucket-sorted order, 64-bit pieces
// per item (run, piece), then map every row through its position (pos1) -> result bits + counts.
#ifndef RPT_BUCKET_UNPERMUTE_THREADS
#define RPT_BUCKET_UNPERMUTE_THREADS 256
#endif
constexpr int kBucketUnpermuteThreads = RPT_BUCKET_UNPERMUTE_THREADS;
__global__ __launch_bounds__(kBucketUnpermuteThreads) void bucket_unpermute_kernel(
    const uint16_t* __restrict__ pos1, const uint64_t* __restrict__ bits2, uint64_t n, uint32_t bucket_mask,
    const uint32_t* __restrict__ counts_tm, const uint32_t* __restrict__ pre_tm, const uint64_t* __restrict__ list_base,
    uint32_t groups, const uint32_t* __restrict__ l1_error, uint64_t* __restrict__ out_bits,
    uint32_t* __restrict__ seg_counts) {
  __shared__ uint32_t s_bits[kL1TileRows / 32];
  __shared__ uint32_t s_start[kMaxBuckets], s_item[kMaxBuckets + 1], s_cnt[kMaxBuckets];
  __shared__ uint64_t s_g[kMaxBuckets];
  __shared__ uint32_t s_wave[kBucketUnpermuteThreads / 64][2];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr uint32_t kWaves = kBucketUnpermuteThreads / 64;
  const uint32_t nb = bucket_mask + 1;
  // XCD-contiguous tiles, as the scatter (same grid): neighbouring tiles' runs are adjacent in their
  // lists, so the 64-bit pass-bit pieces one tile gathers share lines with its neighbours' in the same L2
  const uint64_t tile = l1_tile_of_block(blockIdx.x, gridDim.x);
  const uint64_t* lbase = list_base + static_cast<uint64_t>(l1_group_of_tile(tile, gridDim.x, groups)) * nb;
  const uint64_t n_segs = (n + kSegRows - 1) / kSegRows;
  constexpr uint32_t kSegsPerWave = (kL1TileRows / kSegRows) / kWaves;
  const uint64_t seg0 = tile * (kL1TileRows / kSegRows) + wave * kSegsPerWave;
  u32x4 pv[kSegsPerWave];  // row positions, in flight while the bits are staged
#pragma unroll
  for (uint32_t sg = 0; sg < kSegsPerWave; sg++) {
    pv[sg] = u32x4{0, 0, 0, 0};
    if (seg0 + sg < n_segs) pv[sg] = *reinterpret_cast<const u32x4*>(pos1 + (seg0 + sg) * kSegRows + lane * 8);
  }
  for (uint32_t i = threadIdx.x; i < kL1TileRows / 32; i += kBucketUnpermuteThreads) s_bits[i] = 0;
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
      s_g[b] = lbase[b] + pre_tm[tile * nb + b];
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
  // the scatter hit a bound (never expected): level 2 did not run, every row passes (a Bloom filter may
  // return false positives, never false negatives)
  const bool err = __hip_atomic_load(l1_error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  if (threadIdx.x == 0) s_item[nb] = err ? 0u : total_items;
  __syncthreads();
  for (uint32_t it = threadIdx.x; it < s_item[nb]; it += kBucketUnpermuteThreads) {
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
    for (int c = 0; c < 4; c++) byte |= pass_bits2(s_bits, pv[sg][c]) << (2 * c);
    if (err) byte = 0xFFu;
    const uint64_t row0 = seg * kSegRows + lane * 8;
    if (row0 + 8 > n) byte = row0 >= n ? 0u : byte & ((1u << (n - row0)) - 1u);
    out_bytes[seg * (kSegRows / 8) + lane] = static_cast<uint8_t>(byte);
    const uint32_t cnt = wave_sum(__popc(byte));
    if (lane == 0) seg_counts[seg] = cnt;
  }
}

// B7: after a bucketed insert whose scatter hit a bound (never expected; B1): every filter bit set, so the
// keys it could not insert still pass every probe. Without the flag each workgroup reads one word and leaves.
constexpr int kErrorFillThreads = 256;
__global__ __launch_bounds__(kErrorFillThreads) void l1_error_fill_kernel(uint64_t* __restrict__ words, uint64_t n_words,
                                                                         const uint32_t* __restrict__ l1_error) {
  if (__hip_atomic_load(l1_error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;  // uniform
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kErrorFillThreads + threadIdx.x; i < n_words;
       i += static_cast<uint64_t>(gridDim.x) * kErrorFillThreads)
    words[i] = ~0ULL;
}
}  // namespace rpt
