// bucketed.hpp — level 1 of the bucketed (two-level) strategy for filters of 32 MiB..16 GiB.
// Part of librpt_gpu.so: included by rpt_gpu.hip (one translation unit: kernels and their launches
// stay together without relocatable device code).
#pragma once

namespace rpt {

// ---- bucketed strategy (filters of 2^22..2^31 blocks) ----------------------------------------------
// Level 1 cuts the rows by 32 MiB filter region ("bucket": 256 slices) into one contiguous hash array
// per bucket, each padded to whole 16 Ki-row tiles; level 2 is the partitioned pipeline above over
// those arrays, every bucket against its own 256 slices. bucket = block id >> 22 = hash bits 38...
static_assert(kLogNumMasks + 6 + kSliceLog + kBucketSliceLog <= 40, "level-2 split hashes carry bits 0..39");
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
  const uint64_t tile = blockIdx.x, tile_base = tile * kL1TileRows;
  int64_t wmn = kMinInit, wmx = kMaxInit;
#pragma unroll
  for (int sg = 0; sg < kL1SegsPerWave; sg++) {
    const uint32_t seg_local = wave * (kL1SegsPerWave * kSegRows) + sg * kSegRows;
    uint64_t hh[8];
    bool oo[8];
    int64_t mm[2] = {kMinInit, kMaxInit};
    load_hashes<K, DENSE, MM, RPT_NT_KEY_LOADS>(a, tile_base + seg_local, n, lane, hh, oo, mm);
    if constexpr (MM && KeyTraits<K>::kValues) {
      wave_minmax(mm[0], mm[1]);
      wmn = min(wmn, mm[0]);
      wmx = max(wmx, mm[1]);
    }
#pragma unroll
    for (int j = 0; j < 8; j++)
      if (oo[j]) atomicAdd(&s_cnt[bucket_of(hh[j], bucket_mask)], 1u);
  }
  if constexpr (MM && KeyTraits<K>::kValues) publish_minmax(wmn, wmx, stats);
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
// bucket's run to its place in that bucket's array (index base[b] + pre_tm[tile][b] + i), as the
// level-2 kKeySplit layout: hash bits 0..31 in hash_lo, bits 32..39 in hash_hi. pos_out (u16, probe
// only) records each row's position in the tile's bucket-sorted order.
template <int K, bool DENSE>
__global__ __launch_bounds__(kTileThreads) void bucket_scatter_kernel(KeyArgs a, uint64_t n, uint32_t bucket_mask,
                                                                      const uint32_t* __restrict__ counts_tm,
                                                                      const uint32_t* __restrict__ pre_tm,
                                                                      const uint64_t* __restrict__ base,
                                                                      uint32_t* __restrict__ hash_lo,
                                                                      uint8_t* __restrict__ hash_hi,
                                                                      uint16_t* __restrict__ pos_out) {
  extern __shared__ uint32_t s_lo[];  // kL1TileRows hash words (bits 0..31), bucket-sorted, then
  uint8_t* s_hi = reinterpret_cast<uint8_t*>(s_lo + kL1TileRows);  // their bits 32..39, then
  uint16_t* s_bk = reinterpret_cast<uint16_t*>(s_hi + kL1TileRows);  // their bucket (RPT_SCATTER_FLAT_COPY)
  __shared__ uint32_t s_start[kMaxBuckets], s_cur[kMaxBuckets];
  __shared__ uint64_t s_dst[kMaxBuckets];  // where each bucket's run goes in the level-2 array
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t nb = bucket_mask + 1;
  // Workgroups go round-robin to the 8 XCDs; give each XCD a contiguous range of tiles, so the runs of
  // neighbouring tiles (adjacent in each bucket's array) are written through the same L2 and leave it
  // as whole lines.
  const uint32_t per_xcd = gridDim.x / 8, xcd = blockIdx.x % 8;
  const uint64_t tile = blockIdx.x < per_xcd * 8 ? static_cast<uint64_t>(xcd) * per_xcd + blockIdx.x / 8 : blockIdx.x;
  const uint64_t tile_base = tile * kL1TileRows;
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
  for (int sg = 0; sg < kL1SegsPerWave; sg++) {
    const uint32_t seg_local = wave * (kL1SegsPerWave * kSegRows) + sg * kSegRows;
    const uint64_t sbase = tile_base + seg_local;
    uint64_t hh[8];
    bool oo[8];
    load_hashes<K, DENSE, false, false, true>(a, sbase, n, lane, hh, oo);
    uint16_t pv[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint32_t p = 0;
      if (oo[j]) {
        const uint32_t b = bucket_of(hh[j], bucket_mask);
        p = atomicAdd(&s_cur[b], 1u);
        s_lo[p] = static_cast<uint32_t>(hh[j]);
        s_hi[p] = static_cast<uint8_t>(hh[j] >> 32);
        if (RPT_SCATTER_FLAT_COPY) s_bk[p] = static_cast<uint16_t>(b);
      }
      pv[j] = static_cast<uint16_t>(p);
    }
    if (pos_out != nullptr) {  // padded to whole tiles: rows >= n get don't-care values
#pragma unroll
      for (int j = 0; j < 8; j++) pos_out[sbase + seg_row<K, DENSE>(j, lane)] = pv[j];
    }
  }
  __syncthreads();
  if (RPT_SCATTER_FLAT_COPY) {
    // the tile's bucket-sorted rows in order, every lane busy: a wave's 64 rows span ~2 runs, so each
    // store instruction writes whole pieces of runs (a loop per bucket leaves half the lanes idle)
    for (uint32_t b = threadIdx.x; b < nb; b += kTileThreads) s_dst[b] -= s_start[b];
    __syncthreads();
    const uint32_t used = s_cur[nb - 1];
    for (uint32_t i = threadIdx.x; i < used; i += kTileThreads) {
      const uint64_t d = s_dst[s_bk[i]] + i;
#ifndef RPT_EXP_SCATTER_SKIP
#define RPT_EXP_SCATTER_SKIP 0  // measurement only: 1 = no high-byte stores, 2 = no low-word stores, 3 = neither
#endif
      if (!(RPT_EXP_SCATTER_SKIP & 2)) hash_lo[d] = s_lo[i];
      if (!(RPT_EXP_SCATTER_SKIP & 1)) hash_hi[d] = s_hi[i];
    }
  } else {
    for (uint32_t b = wave; b < nb; b += kTileThreads / 64) {  // LDS only: no global latency in the chain
      const uint32_t c = s_cur[b] - s_start[b], s0 = s_start[b];
      const uint64_t d = s_dst[b];
      for (uint32_t i = lane; i < c; i += 64) {
        hash_lo[d + i] = s_lo[s0 + i];
        hash_hi[d + i] = s_hi[s0 + i];
      }
    }
  }
}

// B5: pad each bucket's array to whole tiles with copies of its first hash (re-inserting or re-probing
// a present hash changes nothing, and the pads' results are never read).
__global__ __launch_bounds__(kBlockThreads) void bucket_pad_kernel(const uint32_t* __restrict__ totals,
                                                                  const uint64_t* __restrict__ base,
                                                                  uint32_t* __restrict__ hash_lo,
                                                                  uint8_t* __restrict__ hash_hi) {
  const uint32_t b = blockIdx.x;
  const uint64_t t = totals[b], b0 = base[b], end = base[b + 1];
  if (t == 0) return;
  const uint32_t lo = hash_lo[b0];
  const uint8_t hi = hash_hi[b0];
  for (uint64_t i = b0 + t + threadIdx.x; i < end; i += kBlockThreads) {
    hash_lo[i] = lo;
    hash_hi[i] = hi;
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
    const uint32_t* __restrict__ counts_tm, const uint32_t* __restrict__ pre_tm, const uint64_t* __restrict__ base,
    uint64_t* __restrict__ out_bits, uint32_t* __restrict__ seg_counts) {
  __shared__ uint32_t s_bits[kL1TileRows / 32];
  __shared__ uint32_t s_start[kMaxBuckets], s_item[kMaxBuckets + 1], s_cnt[kMaxBuckets];
  __shared__ uint64_t s_g[kMaxBuckets];
  __shared__ uint32_t s_wave[kBucketUnpermuteThreads / 64][2];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr uint32_t kWaves = kBucketUnpermuteThreads / 64;
  const uint32_t nb = bucket_mask + 1;
#if RPT_BUCKET_UNPERMUTE_XCD_MAP
  // XCD-contiguous tiles, as the scatter: neighbouring tiles' runs are adjacent in every bucket's array,
  // so the 64-bit pass-bit pieces one tile gathers share lines with its neighbours' in the same L2
  const uint32_t per_xcd = gridDim.x / 8, xcd = blockIdx.x % 8;
  const uint64_t tile = blockIdx.x < per_xcd * 8 ? static_cast<uint64_t>(xcd) * per_xcd + blockIdx.x / 8 : blockIdx.x;
#else
  const uint64_t tile = blockIdx.x;
#endif
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
}  // namespace rpt
