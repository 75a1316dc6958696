// probe_direct.hpp — P1: hash + filter gather (global or whole-filter LDS) -> result bits.
// Part of librpt_gpu.so: included by rpt_gpu.hip (one translation unit: kernels and their launches
// stay together without relocatable device code).
#pragma once

namespace rpt {

// ---- P1: probe -> result bits + per-segment survivor counts ------------------------------------
// FILTER_IN_LDS: the whole filter (<= 128 KiB) is staged in LDS and every gather is an LDS read; it runs
// 1024-thread workgroups (kLdsProbeThreads).
//
// Full segments of flat columns without validity take a software-pipelined loop: the wave's next
// segments are loaded into a second set of registers (ping-pong, so no register copy has to wait for
// them) while the current ones are hashed and probed. The general loop (load_hashes: tails, validity,
// dictionaries) takes whatever is left.
#ifndef RPT_NT_PROBE_LOADS
#define RPT_NT_PROBE_LOADS 1  // non-temporal key loads in the pipelined direct probes (128 KiB LDS probe 1.69 -> 1.56 ms per 1e9 int64 keys)
#endif
#ifndef RPT_PROBE_PREFETCH
#define RPT_PROBE_PREFETCH 2  // segments per prefetched group (0: off)
#endif
#ifndef RPT_LDS_I64_GROUP
#define RPT_LDS_I64_GROUP 1  // segments per group in the int64 whole-filter LDS probe (r02: 2 and 3 were slower)
#endif
#ifndef RPT_PROBE_SCHED_BARRIER
#define RPT_PROBE_SCHED_BARRIER 0  // 1: scheduling barrier after the prefetch loads (measured: no gain, see the loop)
#endif
#ifndef RPT_HYBRID_I64_GROUP
#define RPT_HYBRID_I64_GROUP 2  // segments per group in the int64 hybrid LDS/L2 probe (1 / 2 / 3: 2.82 / 2.59 / 2.87 ms
                                // per 1e9 keys, profiles/r06/ab_hybrid_group.txt; int32 takes RPT_PROBE_PREFETCH = 2)
#endif
#ifndef RPT_PROBE_RING
#define RPT_PROBE_RING 2  // register buffers of prefetched groups: 2 = ping-pong (group g + 1 in flight while g is
                          // probed), 3 = groups g + 1 and g + 2 in flight
#endif
template <int K> struct RawSeg {
  static constexpr int V = KeyTraits<K>::kVec;
  static constexpr int kLoads = 8 / V;
  using Vec = typename std::conditional<V == 2, u64x2, u32x4>::type;
  Vec r[kLoads];
  __device__ __forceinline__ void load(const void* keys, uint64_t seg, uint32_t lane) {
    using T = typename KeyTraits<K>::T;
    const T* kb = static_cast<const T*>(keys) + seg * kSegRows + lane * V;
#pragma unroll
    for (int c = 0; c < kLoads; c++) r[c] = stream_load<RPT_NT_PROBE_LOADS>(reinterpret_cast<const Vec*>(kb + c * 64 * V));
  }
  __device__ __forceinline__ void hashes(uint64_t (&h)[8]) const {
    using T = typename KeyTraits<K>::T;
#pragma unroll
    for (int c = 0; c < kLoads; c++)
#pragma unroll
      for (int e = 0; e < V; e++) h[c * V + e] = KeyTraits<K>::hash(static_cast<T>(r[c][e]));
  }
};

// HYBRID (filters of 256 KiB .. 2^RPT_LDS_HYBRID_MAX_LOG blocks): the filter's first kHybridWords words are staged in
// LDS, the rest gathered from L2.
constexpr uint64_t kHybridWords = 1ULL << kLdsDirectMaxLog;
template <bool FILTER_IN_LDS, bool HYBRID = false>
__device__ __forceinline__ void probe8(const uint64_t* __restrict__ words, const uint64_t* s_filter,
                                       const uint64_t* s_masks, uint64_t block_mask, const uint64_t (&h)[8],
                                       const bool (&ok)[8], bool (&pass)[8]) {
  uint64_t w[8], m[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    m[j] = mask_of(s_masks, h[j]);
    if constexpr (FILTER_IN_LDS && HYBRID) {
      const uint64_t blk = block_of(h[j], block_mask);
      w[j] = blk < kHybridWords ? s_filter[blk] : (ok[j] ? words[blk] : 0ULL);
    } else if constexpr (FILTER_IN_LDS) {
      w[j] = s_filter[block_of(h[j], block_mask)];
    } else {
      w[j] = ok[j] ? words[block_of(h[j], block_mask)] : 0ULL;
    }
  }
#pragma unroll
  for (int j = 0; j < 8; j++) pass[j] = ok[j] && (w[j] & m[j]) == m[j];
}

// zero[0 .. n_zero): words the selection-vector tail's look-back needs cleared (compact_lookback_kernel's group
// states and ticket), cleared here so the tail needs no launch of its own; nullptr when there is no such tail.
// The body of probe_bits_kernel (HYBRID = false) and probe_bits_hybrid_kernel (HYBRID = true: filters of 256 KiB,
// the first 128 KiB staged in LDS, the rest gathered from L2).
template <int K, bool DENSE, bool FILTER_IN_LDS, int THREADS, bool HYBRID>
__device__ __forceinline__ void probe_bits_body(const uint64_t* __restrict__ words, uint64_t block_mask, KeyArgs a,
                                                uint64_t n, uint64_t n_segs, uint64_t* __restrict__ out_bits,
                                                uint32_t* __restrict__ seg_counts, uint64_t* __restrict__ zero,
                                                uint32_t n_zero) {
  __shared__ uint64_t s_masks[kNumMasks];
  extern __shared__ uint64_t s_filter[];
  for (uint32_t i = blockIdx.x * THREADS + threadIdx.x; i < n_zero; i += gridDim.x * THREADS) zero[i] = 0;
  fill_mask_table(s_masks);
  if constexpr (FILTER_IN_LDS) {
    const uint64_t staged = HYBRID ? kHybridWords - 1 : block_mask;
    for (uint64_t i = threadIdx.x; i <= staged; i += blockDim.x) s_filter[i] = words[i];
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  constexpr uint32_t kWaves = THREADS / 64;
  const uint64_t total_waves = static_cast<uint64_t>(gridDim.x) * kWaves;
  // the wave index is uniform: keep seg in scalar registers
  uint64_t seg = static_cast<uint64_t>(blockIdx.x) * kWaves +
                 static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)));
#if RPT_PROBE_PREFETCH
  if constexpr (DENSE && K != kKeySplit) {
    const uint64_t n_full = n / kSegRows;
    if (a.validity == nullptr && seg < n_full) {
      // groups of S segments (seg, seg + tw, ...); a group's loads are issued before the previous
      // group is probed. Addresses past the last full segment are clamped and their rows discarded.
      // measured (ms per 1e9 keys, S = 1 / 2 / 3): 128 KiB LDS int64 1.68 / 1.79 / 1.77, int32 1.09 /
      // 1.05 / 1.06; 256 KiB gather 4.48 / 4.33 / 4.30
      constexpr int S = (FILTER_IN_LDS && KeyTraits<K>::kVec == 2) ? (HYBRID ? RPT_HYBRID_I64_GROUP : RPT_LDS_I64_GROUP)
                                                                   : RPT_PROBE_PREFETCH;
      constexpr int NB = RPT_PROBE_RING;
      const bool ok[8] = {true, true, true, true, true, true, true, true};
      const uint64_t first = seg;
      RawSeg<K> R[NB][S];
      auto load_group = [&](RawSeg<K>(&R)[S], uint64_t g) {
#pragma unroll
        for (int q = 0; q < S; q++) {
          const uint64_t sg = g + q * total_waves;
          R[q].load(a.keys, sg < n_full ? sg : n_full - 1, lane);
        }
      };
      auto probe_group = [&](const RawSeg<K>(&R)[S], uint64_t g) {
#pragma unroll
        for (int q = 0; q < S; q++) {
          const uint64_t sg = g + q * total_waves;
          if (sg < n_full) {
            uint64_t h[8];
            bool pass[8];
#if defined(RPT_EXP_PROBE_NO_HASH)  // measurement only: pass = a key bit (no hash, no filter lookups)
#pragma unroll
            for (int c = 0; c < RawSeg<K>::kLoads; c++)
#pragma unroll
              for (int e = 0; e < RawSeg<K>::V; e++) pass[c * RawSeg<K>::V + e] = (R[q].r[c][e] >> 7) & 1;
            (void)h;
#elif defined(RPT_EXP_PROBE_NO_LDS)  // measurement only: pass = a hash bit (hash kept, no filter lookups)
            R[q].hashes(h);
#pragma unroll
            for (int j = 0; j < 8; j++) pass[j] = (h[j] >> 21) & 1;
#else
            R[q].hashes(h);
            probe8<FILTER_IN_LDS, HYBRID>(words, s_filter, s_masks, block_mask, h, ok, pass);
#endif
            store_segment_bits<K, DENSE, RPT_PROBE_BUFSTORE>(pass, lane, sg, out_bits, seg_counts);
          }
        }
      };
      const uint64_t step = S * total_waves;
#pragma unroll
      for (int b = 0; b < NB - 1; b++) load_group(R[b], seg + b * step);
      bool more = true;
      while (more) {
        // buffer b holds group seg; before probing it, the group NB - 1 steps ahead goes into the buffer the
        // previous iteration freed (compile-time indices: the loop over b is unrolled)
#pragma unroll
        for (int b = 0; b < NB; b++) {
          if (more) {
            load_group(R[(b + NB - 1) % NB], seg + (NB - 1) * step);
            asm volatile("" ::: "memory");  // issue the next group's loads before this one's work
#if RPT_PROBE_SCHED_BARRIER
            // ... and keep the scheduler from hoisting this group's hashing above them: it does in the second half of
            // the unrolled int64 ping-pong, whose wait for its data then finds no loads in flight. Pinning the order
            // measured no faster (profiles/r06/ab_pipeline.txt): 16 waves per CU hide that wait.
            __builtin_amdgcn_sched_barrier(0);
#endif
            probe_group(R[b], seg);
            seg += step;
            more = seg < n_full;
          }
        }
      }
      // the general loop resumes at this wave's first segment past the full ones
      seg = first + (n_full - first + total_waves - 1) / total_waves * total_waves;
    }
  }
#endif
  for (; seg < n_segs; seg += total_waves) {
    uint64_t h[8];
    bool ok[8], pass[8];
    load_hashes<K, DENSE>(a, seg * kSegRows, n, lane, h, ok);
    probe8<FILTER_IN_LDS, HYBRID>(words, s_filter, s_masks, block_mask, h, ok, pass);
    store_segment_bits<K, DENSE>(pass, lane, seg, out_bits, seg_counts);
  }
}

template <int K, bool DENSE, bool FILTER_IN_LDS, int THREADS = kBlockThreads>
__global__ __launch_bounds__(THREADS) void probe_bits_kernel(const uint64_t* __restrict__ words,
                                                                  uint64_t block_mask, KeyArgs a, uint64_t n,
                                                                  uint64_t n_segs, uint64_t* __restrict__ out_bits,
                                                                  uint32_t* __restrict__ seg_counts,
                                                                  uint64_t* __restrict__ zero, uint32_t n_zero) {
  probe_bits_body<K, DENSE, FILTER_IN_LDS, THREADS, false>(words, block_mask, a, n, n_segs, out_bits, seg_counts, zero,
                                                           n_zero);
}
template <int K, bool DENSE>
__global__ __launch_bounds__(kLdsProbeThreads) void probe_bits_hybrid_kernel(const uint64_t* __restrict__ words,
                                                                             uint64_t block_mask, KeyArgs a, uint64_t n,
                                                                             uint64_t n_segs, uint64_t* __restrict__ out_bits,
                                                                             uint32_t* __restrict__ seg_counts,
                                                                             uint64_t* __restrict__ zero, uint32_t n_zero) {
  probe_bits_body<K, DENSE, true, kLdsProbeThreads, true>(words, block_mask, a, n, n_segs, out_bits, seg_counts, zero,
                                                          n_zero);
}

// ---- small batches: probe + compaction in ONE workgroup ----------------------------------------
// A DuckDB-sized call (one to eight 2048-row vectors) is dominated by launch and copy latency, not by
// bytes: probe_bits + group_sum + group_scan + compact become one launch of one workgroup. Each wave
// probes whole 512-row segments (gathers from the L2-resident filter) into row-ordered result words
// in LDS, then the segments' counts are scanned and every wave expands its segments' words into the
// ascending selection vector. n <= kSmallRows.
constexpr int kSmallThreads = 1024;
constexpr uint64_t kSmallRows = RPT_SMALL_PROBE_ROWS;
// Every 512-row segment is some wave's (probe_small_kernel's kPerWave = segments / waves must not round
// down: a dropped segment would drop its rows) and small_sel_tail's one-wave scan covers every segment count.
static_assert(kSmallRows % (kSegRows * (kSmallThreads / 64)) == 0 && kSmallRows / kSegRows <= 64,
              "RPT_SMALL_PROBE_ROWS must be a multiple of 8192 rows, at most 32768");
// The small kernels' tail: segment counts (<= 32) -> the ascending selection vector. Every wave scans the
// counts itself (lane i holds segment i's) and expands its own segments' row-ordered result words.
__device__ __forceinline__ void small_sel_tail(const uint64_t* s_words, const uint32_t* s_cnt, uint32_t n_segs,
                                               const uint32_t* __restrict__ row_sel, uint32_t* __restrict__ out_sel,
                                               uint64_t* __restrict__ out_count) {
  constexpr uint32_t kWaves = kSmallThreads / 64;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t c = lane < n_segs ? s_cnt[lane] : 0u;
  const uint32_t incl = wave_inclusive_sum(c);
  if (threadIdx.x == 0) *out_count = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), 63));
  for (uint32_t seg = wave; seg < n_segs; seg += kWaves) {
    // lanes 0..7 own the segment's 8 result words (64 rows each); pc = their survivors
    uint64_t word = lane < kWordsPerSeg ? s_words[seg * kWordsPerSeg + lane] : 0ULL;
    const uint32_t pc = __popcll(word);
    uint32_t p = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl - c), static_cast<int>(seg))) +
                 wave_inclusive_sum(pc) - pc;
    const uint32_t row0 = seg * static_cast<uint32_t>(kSegRows) + lane * 64;
    while (word) {
      const uint32_t row = row0 + __builtin_ctzll(word);
      out_sel[p++] = row_sel ? row_sel[row] : row;
      word &= word - 1;
    }
  }
}

template <int K, bool DENSE>
__global__ __launch_bounds__(kSmallThreads) void probe_small_kernel(const uint64_t* __restrict__ words,
                                                                   uint64_t block_mask, KeyArgs a, uint64_t n,
                                                                   const uint32_t* __restrict__ row_sel,
                                                                   uint32_t* __restrict__ out_sel,
                                                                   uint64_t* __restrict__ out_count) {
  constexpr uint32_t kSegs = kSmallRows / kSegRows;
  constexpr uint32_t kWaves = kSmallThreads / 64;
  __shared__ uint64_t s_masks[kNumMasks];
  __shared__ uint64_t s_words[kSegs * kWordsPerSeg];
  __shared__ uint32_t s_cnt[kSegs];
  fill_mask_table(s_masks);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t n_segs = static_cast<uint32_t>((n + kSegRows - 1) / kSegRows);
  // a wave's segments (<= kSegs / kWaves) are all loaded before any is probed: the keys usually sit in
  // device-mapped host memory, one PCIe round trip per dependent load
  constexpr uint32_t kPerWave = kSegs / kWaves;
  uint64_t h[kPerWave][8];
  bool ok[kPerWave][8];
#pragma unroll
  for (uint32_t i = 0; i < kPerWave; i++) {
    const uint32_t seg = wave + i * kWaves;
    if (seg < n_segs) load_hashes<K, DENSE>(a, static_cast<uint64_t>(seg) * kSegRows, n, lane, h[i], ok[i]);
  }
#pragma unroll
  for (uint32_t i = 0; i < kPerWave; i++) {
    const uint32_t seg = wave + i * kWaves;
    if (seg >= n_segs) break;
    bool pass[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint64_t m = mask_of(s_masks, h[i][j]);
      const uint64_t w = ok[i][j] ? words[block_of(h[i][j], block_mask)] : 0ULL;
      pass[j] = ok[i][j] && (w & m) == m;
    }
    store_segment_bits<K, DENSE>(pass, lane, seg, s_words, s_cnt);
  }
  __syncthreads();
  small_sel_tail(s_words, s_cnt, n_segs, row_sel, out_sel, out_count);
}

// ---- USE_BF's filter chain in one launch -----------------------------------------------------------
// PhysicalUseBF::ExecuteInternal (physical_use_bf.cpp:127-179) runs its filters one after another, each
// LookupSel over the rows the previous ones kept, so its result is the AND of the filters.
// For a DuckDB-sized batch each LookupSel is latency-bound (launch, sync, and the key loads: the host
// mirror passes device-mapped pinned host memory, one PCIe round trip), so the whole chain is one
// single-workgroup launch whose (filter, 512-row segment) probes are independent items spread over the
// 16 waves: every filter's key loads and gathers are in flight at once instead of one filter after
// another (rows already failed are probed anyway: a gather costs less than the round trip it would
// wait for). Each item's pass words land in LDS; their AND per word becomes the sel as in
// probe_small_kernel. Columns of different key types share the general row mapping (row = base + 64 c +
// lane). k <= kMaxChain, n <= kSmallRows.
constexpr uint32_t kMaxChain = RPT_MAX_CHAIN;
struct ChainArgs {
  const uint64_t* words[kMaxChain];
  uint64_t block_mask[kMaxChain];
  KeyArgs a[kMaxChain];
  int32_t key_type[kMaxChain];
  uint32_t k;
};
// The hashes of a lane's 8 rows of a segment in the general mapping. Unlike load_hashes' general path
// (a branch per row around dependent loads), the selection lookups are uniform branches and each level's
// 8 loads are issued back to back: the keys usually sit in device-mapped host memory, where every
// dependent load is a PCIe round trip (8 serialized key loads made the chain kernel 17 us, not 3).
template <int K>
__device__ __forceinline__ void chain_hashes(const KeyArgs& a, uint64_t base, uint64_t n, uint32_t lane,
                                             uint64_t (&h)[8], bool (&ok)[8]) {
  using Tr = KeyTraits<K>;
  using T = typename Tr::T;
  const uint32_t rem = static_cast<uint32_t>(n - base < kSegRows ? n - base : kSegRows);  // base < n
  uint64_t idx[8];
#pragma unroll
  for (int c = 0; c < 8; c++) {
    const uint32_t off = static_cast<uint32_t>(c * 64) + lane;
    ok[c] = off < rem;
    idx[c] = base + (ok[c] ? off : 0u);  // rows past n read row `base` (in range) and are discarded
  }
  if (a.row_sel != nullptr) {
#pragma unroll
    for (int c = 0; c < 8; c++) idx[c] = a.row_sel[idx[c]];
  }
  if (a.key_sel != nullptr) {
#pragma unroll
    for (int c = 0; c < 8; c++) idx[c] = a.key_sel[idx[c]];
  }
  const T* keys = static_cast<const T*>(a.keys);
  T kv[8];
#pragma unroll
  for (int c = 0; c < 8; c++) kv[c] = keys[idx[c]];
  uint64_t vw[8];
#pragma unroll
  for (int c = 0; c < 8; c++) vw[c] = ~0ULL;
  if (Tr::kValues && a.validity != nullptr) {
#pragma unroll
    for (int c = 0; c < 8; c++) vw[c] = a.validity[idx[c] >> 6];
  }
#pragma unroll
  for (int c = 0; c < 8; c++) {
    uint64_t hv = Tr::hash(kv[c]);
    if (Tr::kValues && !((vw[c] >> (idx[c] & 63)) & 1ULL)) hv = kNullHash;
    h[c] = hv;
  }
}
template <int K>
__device__ __forceinline__ void chain_probe(const KeyArgs& a, const uint64_t* __restrict__ words, uint64_t block_mask,
                                            const uint64_t* s_masks, uint64_t base, uint64_t n, uint32_t lane,
                                            bool (&pass)[8]) {
  uint64_t h[8];
  bool ok[8];
  chain_hashes<K>(a, base, n, lane, h, ok);
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const uint64_t m = mask_of(s_masks, h[j]);
    const uint64_t w = ok[j] ? words[block_of(h[j], block_mask)] : 0ULL;
    pass[j] = ok[j] && (w & m) == m;
  }
}
__global__ __launch_bounds__(kSmallThreads) void probe_chain_small_kernel(ChainArgs c, uint64_t n,
                                                                          const uint32_t* __restrict__ row_sel,
                                                                          uint32_t* __restrict__ out_sel,
                                                                          uint64_t* __restrict__ out_count) {
  constexpr uint32_t kSegs = kSmallRows / kSegRows;
  constexpr uint32_t kWaves = kSmallThreads / 64;
  __shared__ uint64_t s_masks[kNumMasks];
  __shared__ uint64_t s_pass[kMaxChain][kSegs * kWordsPerSeg];  // each filter's row-ordered pass words
  __shared__ uint64_t s_words[kSegs * kWordsPerSeg];
  __shared__ uint32_t s_cnt[kSegs];
  fill_mask_table(s_masks);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t n_segs = static_cast<uint32_t>((n + kSegRows - 1) / kSegRows);
  for (uint32_t it = wave; it < c.k * n_segs; it += kWaves) {
    const uint32_t f = it / n_segs, seg = it - f * n_segs;  // uniform
    const uint64_t base = static_cast<uint64_t>(seg) * kSegRows;
    bool pass[8];
    if (c.key_type[f] == kKeyI64) chain_probe<kKeyI64>(c.a[f], c.words[f], c.block_mask[f], s_masks, base, n, lane, pass);
    else if (c.key_type[f] == kKeyI32) chain_probe<kKeyI32>(c.a[f], c.words[f], c.block_mask[f], s_masks, base, n, lane, pass);
    else chain_probe<kKeyHash>(c.a[f], c.words[f], c.block_mask[f], s_masks, base, n, lane, pass);
    store_segment_bits<kKeyI64, false>(pass, lane, seg, s_pass[f], nullptr);
  }
  __syncthreads();
  // the AND over the filters, word by word; then each segment's survivor count
  for (uint32_t w = threadIdx.x; w < n_segs * kWordsPerSeg; w += kSmallThreads) {
    uint64_t x = s_pass[0][w];
    for (uint32_t f = 1; f < c.k; f++) x &= s_pass[f][w];
    s_words[w] = x;
  }
  __syncthreads();
  for (uint32_t seg = wave; seg < n_segs; seg += kWaves) {
    const uint32_t pc = lane < kWordsPerSeg ? static_cast<uint32_t>(__popcll(s_words[seg * kWordsPerSeg + lane])) : 0u;
    const uint32_t t = wave_sum(pc);
    if (lane == 0) s_cnt[seg] = t;
  }
  __syncthreads();
  small_sel_tail(s_words, s_cnt, n_segs, row_sel, out_sel, out_count);
}
}  // namespace rpt
