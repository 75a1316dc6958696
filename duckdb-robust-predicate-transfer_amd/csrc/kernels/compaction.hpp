// compaction.hpp — P2/P3: result bits -> ascending uint32 selection vector.
// Part of librpt_gpu.so: included by rpt_gpu.hip (one translation unit: kernels and their launches
// stay together without relocatable device code).
#pragma once

namespace rpt {

// ---- P2a: survivor count per group of kGroupSegs (256) segments --------------------------------------------
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

// ---- P2a + P2b in one launch (direct strategies; RPT_SUMSCAN_TAIL=1, off) -------------------------
// group_sum_kernel's work, after which the highest-numbered workgroup scans the group sums as group_scan_kernel
// does: one dependent launch fewer. Built because a kernel trace showed ~10 us of idle GPU before each dependent
// launch (profiles/r06/jobdim_kernel_gaps.txt) -- but those gaps were the profiling events' own: without them the
// step's kernels run back to back (profiles/r06/kernel_events_overhead.txt), and this kernel (0.024 ms with the
// scan's tile in registers, 0.030-0.035 with this LDS-staged tile) is slower than the two it replaces (0.016 ms),
// so it stays off. state[g] = kSumValid | group g's sum; the probe kernel cleared the words and the scanning workgroup clears them again as it reads them (a repeated
// phase 2 also works). Workgroups are dispatched in index order, so when the last one runs every other one is
// running or done and its wait is short. Measured on the way (tools/ubench/ubench_sumscan.hip,
// profiles/r06/ubench_sumscan.txt): a release per workgroup (an L2 write-back) made the kernel 0.17 ms, and a
// "last workgroup done" counter 0.09 ms more (7630 same-address atomics serialize at ~12 ns each), against 0.007
// for the sums alone. Each sum carries its own valid bit, so relaxed agent-scope atomics suffice; the scanning
// workgroup reads them with atomic exchanges (performed at the coherence point, and clearing as they read), and a
// sum still invalid after kSumSpins polls is recomputed from the segment counts (correct, slow, never a hang).
#ifndef RPT_SCAN_ROWS
#define RPT_SCAN_ROWS 32
#endif
constexpr uint32_t kScanRows = RPT_SCAN_ROWS;  // the scanning workgroup's tiles: kScanRows x 256 group sums in LDS
constexpr uint32_t kSumValid = 1u << 31, kSumSpins = 1u << 12;
__global__ __launch_bounds__(kBlockThreads) void group_sum_scan_kernel(const uint32_t* __restrict__ seg_counts,
                                                                      uint64_t n_segs, uint32_t n_groups,
                                                                      uint32_t* __restrict__ state,
                                                                      uint32_t* __restrict__ group_offs,
                                                                      uint64_t* __restrict__ out_count) {
  static_assert(kGroupSegs == kBlockThreads, "one segment count per thread");
  constexpr uint32_t kTile = kScanRows * kBlockThreads;
  __shared__ uint32_t s_part[kWavesPerBlock];
  __shared__ uint32_t s_wt[kWavesPerBlock][kScanRows];
  __shared__ uint32_t s_tile[kTile];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kGroupSegs + threadIdx.x;
  uint32_t s = i < n_segs ? seg_counts[i] : 0u;
  s = wave_sum(s);
  if (lane == 0) s_part[wave] = s;
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store(state + blockIdx.x, kSumValid | (s_part[0] + s_part[1] + s_part[2] + s_part[3]),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (blockIdx.x != n_groups - 1) return;
  // tile element (row k, thread t) is group base + k * 256 + t: all of a tile's exchanges are in flight at once;
  // the scan runs along rows (one wave scan per row) then down the row totals
  uint32_t carry = 0;
  for (uint32_t base = 0; base < n_groups; base += kTile) {
#pragma unroll
    for (uint32_t k = 0; k < kScanRows; k++) {
      const uint32_t g = base + k * kBlockThreads + threadIdx.x;
      s_tile[k * kBlockThreads + threadIdx.x] =
          g < n_groups ? __hip_atomic_exchange(state + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kSumValid;
    }
    // sums not visible yet (rare): wait for them, bounded, then recompute from the segment counts
    for (uint32_t k = 0; k < kScanRows; k++) {
      const uint32_t g = base + k * kBlockThreads + threadIdx.x;
      uint32_t v = s_tile[k * kBlockThreads + threadIdx.x];
      if (v & kSumValid) continue;
      for (uint32_t spins = 0; !(v & kSumValid) && spins < kSumSpins; spins++) {
        __builtin_amdgcn_s_sleep(1);
        v = __hip_atomic_exchange(state + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (!(v & kSumValid)) {
        uint32_t c = 0;
        for (uint64_t q = static_cast<uint64_t>(g) * kGroupSegs; q < n_segs && q < (g + 1ULL) * kGroupSegs; q++)
          c += seg_counts[q];
        v = kSumValid | c;
      }
      s_tile[k * kBlockThreads + threadIdx.x] = v;
    }
    // row totals per wave first, the rows' wave scans again afterwards (recomputing 6 DPP adds per row instead of
    // holding 32 more registers: this kernel's register count sets the occupancy of its short sum phase)
#pragma unroll
    for (uint32_t k = 0; k < kScanRows; k++) {
      const uint32_t tot = wave_sum(s_tile[k * kBlockThreads + threadIdx.x] & ~kSumValid);
      if (lane == 0) s_wt[wave][k] = tot;
    }
    __syncthreads();
    uint32_t row_base = carry;
#pragma unroll
    for (uint32_t k = 0; k < kScanRows; k++) {
      const uint32_t v = s_tile[k * kBlockThreads + threadIdx.x] & ~kSumValid;
      uint32_t before = 0;
      for (uint32_t w = 0; w < wave; w++) before += s_wt[w][k];
      const uint32_t g = base + k * kBlockThreads + threadIdx.x;
      if (g < n_groups) group_offs[g] = row_base + before + wave_inclusive_sum(v) - v;
      row_base += s_wt[0][k] + s_wt[1][k] + s_wt[2][k] + s_wt[3][k];
    }
    carry = row_base;
    __syncthreads();
  }
  if (threadIdx.x == 0) *out_count = carry;
}

// ---- P3: expand result bits into an ascending selection vector ----------------------------------
// Entries of each wave's staging buffer. 8 * RPT_COMPACT_BALLOT_MIN (3072, 6 KiB per wave) rather than a whole
// step's 4096 rows: 24 KiB of LDS per workgroup lets 6 workgroups share a CU instead of 4 (the kernel waits on
// its stores and LDS, so more waves hide more): C5 compaction 0.153-0.154 -> 0.130 ms at p = 0.1, 0.468 ->
// 0.426-0.430 ms at p = 0.5 (profiles/r05/ab_compact_stage.txt)
#ifndef RPT_COMPACT_STAGE
#define RPT_COMPACT_STAGE (RPT_SEL_BALLOT_EXPAND ? 8 * RPT_COMPACT_BALLOT_MIN : 8 * 512)
#endif
constexpr uint32_t kCompactStage = RPT_COMPACT_STAGE;
// RPT_COMPACT_V16 = 1: sparse steps write their staged survivors as 16-B units aligned to the destination (4-B
// stores only at the region's two ends) instead of one 4-B store per lane. A plain 4-B-per-lane write stream runs
// at 4.4 TB/s, a 16-B one at 6.6, and compact's region pattern gains 0.01 ms from them with placeholder values
// (tools/ubench/ubench_compact.hip) -- but the kernel itself measured 0.155-0.159 vs 0.147-0.152 ms with them
// (profiles/r06/ab_compact_v16.txt), so off.
#ifndef RPT_COMPACT_V16
#define RPT_COMPACT_V16 0
#endif
// a staging row holds kCompactStage survivors behind up to 3 entries of alignment shift
constexpr uint32_t kCompactStageRow = kCompactStage + (RPT_COMPACT_V16 ? 4 : 0);
static_assert(kCompactStage == 8 * kSegRows || (RPT_SEL_BALLOT_EXPAND && kCompactStage >= 8 * RPT_COMPACT_BALLOT_MIN),
              "the LDS staging must hold every sparse step's survivors");
// Group `group`'s 256 segments expanded into the sel, given the group's sel offset (s_off: every segment's offset,
// filled by the caller); every wave of the workgroup calls it.
__device__ __forceinline__ void compact_group(const uint64_t* __restrict__ bits, uint64_t n_segs, uint64_t group,
                                              const uint32_t* s_off, uint16_t (*s_stage)[kCompactStageRow],
                                              const uint32_t* __restrict__ row_sel, uint32_t* __restrict__ out_sel);

__global__ __launch_bounds__(kBlockThreads) void compact_kernel(const uint64_t* __restrict__ bits,
                                                               const uint32_t* __restrict__ seg_counts, uint64_t n_segs,
                                                               const uint32_t* __restrict__ group_offs,
                                                               const uint32_t* __restrict__ row_sel,
                                                               uint32_t* __restrict__ out_sel) {
  __shared__ uint32_t s_off[kGroupSegs];
  __shared__ uint32_t s_wave[kWavesPerBlock];
  // one 4096-row step's survivors per wave (row offsets); a step only stages when it has fewer than
  // 8 * RPT_COMPACT_BALLOT_MIN survivors (denser steps expand word by word), so that many entries suffice
  __shared__ __attribute__((aligned(16))) uint16_t s_stage[kWavesPerBlock][kCompactStageRow];
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
  compact_group(bits, n_segs, blockIdx.x, s_off, s_stage, row_sel, out_sel);
}

// ---- P2 + P3 in one launch: the groups' sel offsets by a decoupled look-back ------------------------
// The direct probes' tail (gather / whole-filter LDS strategies) without group_sum_kernel and group_scan_kernel:
// each workgroup takes the next group in order from a ticket counter (so every group it waits on belongs to a
// workgroup that is already running), sums its 256 segment counts, publishes that aggregate at once, then walks
// back over its predecessors' states 64 at a time (one wave) until it meets an inclusive prefix. A group's
// aggregate needs only its 1 KiB of counts, so the predecessors publish within microseconds and the walk is short.
// state[g]: bits 62-63 = 1 (aggregate) / 2 (inclusive prefix), bits 0-61 = the value; state[n_groups] = the
// ticket counter. The probe kernel that wrote the counts zeroed them (phase 1), so no extra launch clears them.
// Every wait is bounded: a walk that does not complete in kLookbackSpins polls falls back to summing its
// predecessors' segment counts itself (correct, slow, never a hang).
#ifndef RPT_LB_TICKET
#define RPT_LB_TICKET 1  // groups taken from a ticket counter (1) or by blockIdx (0)
#endif
constexpr uint64_t kLbAgg = 1ULL << 62, kLbIncl = 2ULL << 62, kLbValue = (1ULL << 62) - 1;
constexpr uint32_t kLookbackSpins = 1u << 16;
// A state word carries its own value, so relaxed device-scope atomics suffice: nothing else is published with it.
// (Release / acquire at agent scope would write back / invalidate the XCD's L2 on every publish and poll: a
// first version with them took 0.95 ms instead of 0.15.)
__device__ __forceinline__ uint64_t lb_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
  for (int d = 32; d >= 1; d >>= 1) v += static_cast<uint64_t>(__shfl_xor(static_cast<unsigned long long>(v), d, 64));
  return v;
}
__global__ __launch_bounds__(kBlockThreads) void compact_lookback_kernel(const uint64_t* __restrict__ bits,
                                                                        const uint32_t* __restrict__ seg_counts,
                                                                        uint64_t n_segs, uint32_t n_groups,
                                                                        uint64_t* __restrict__ state,
                                                                        const uint32_t* __restrict__ row_sel,
                                                                        uint32_t* __restrict__ out_sel,
                                                                        uint64_t* __restrict__ out_count) {
  __shared__ uint32_t s_off[kGroupSegs];
  __shared__ uint32_t s_wave[kWavesPerBlock];
  __shared__ __attribute__((aligned(16))) uint16_t s_stage[kWavesPerBlock][kCompactStageRow];
  __shared__ uint32_t s_group;
  __shared__ uint64_t s_prefix;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#if RPT_LB_TICKET
  if (threadIdx.x == 0)
    s_group = __hip_atomic_fetch_add(reinterpret_cast<uint32_t*>(state + n_groups), 1u, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const uint32_t g = s_group;
#else
  // workgroups are dispatched in blockIdx order, so every group a workgroup waits on is already running (and the
  // bounded wait would fall back to a direct sum if that ever failed)
  const uint32_t g = blockIdx.x;
  (void)s_group;
#endif
  const uint64_t sidx = static_cast<uint64_t>(g) * kGroupSegs + threadIdx.x;
  const uint32_t c = sidx < n_segs ? seg_counts[sidx] : 0u;
  const uint32_t incl = wave_inclusive_sum(c);
  if (lane == 63) s_wave[wave] = incl;
  __syncthreads();
  if (wave == 0) {
    const uint64_t total = static_cast<uint64_t>(s_wave[0]) + s_wave[1] + s_wave[2] + s_wave[3];
    if (lane == 0)
      lb_store(state + g, (g == 0 ? kLbIncl : kLbAgg) | total);
    uint64_t prefix = 0;
    if (g > 0) {
      int64_t top = static_cast<int64_t>(g) - 1;  // the window is groups top - 63 .. top, lane l reads top - l
      uint32_t spins = 0;
      bool done = false;
      while (!done) {
        const int64_t idx = top - static_cast<int64_t>(lane);
        const uint64_t v = idx >= 0 ? lb_load(state + idx) : kLbIncl;  // before group 0: an inclusive 0
        const uint64_t incl_mask = __ballot((v & ~kLbValue) == kLbIncl);
        const uint64_t ready_mask = __ballot((v & ~kLbValue) != 0);
        // lanes up to the nearest inclusive prefix (all 64 if none) must have published
        const uint64_t need = incl_mask ? (incl_mask & (0ULL - incl_mask)) * 2 - 1 : ~0ULL;
        if ((ready_mask & need) != need) {
          if (++spins >= kLookbackSpins) break;  // fall back below
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        prefix += wave_sum64(((need >> lane) & 1) ? (v & kLbValue) : 0);
        if (incl_mask) done = true;
        else top -= 64;
      }
      if (!done) {  // bounded wait exceeded: sum every predecessor's segment counts directly
        uint64_t s = 0;
        for (uint64_t i = lane; i < static_cast<uint64_t>(g) * kGroupSegs; i += 64) s += seg_counts[i];
        prefix = wave_sum64(s);
      }
      if (lane == 0)
        lb_store(state + g, kLbIncl | (prefix + total));
    }
    if (lane == 0) {
      s_prefix = prefix;
      if (g == n_groups - 1) *out_count = prefix + total;
    }
  }
  __syncthreads();
  uint32_t off = static_cast<uint32_t>(s_prefix) + incl - c;
  for (uint32_t w = 0; w < wave; w++) off += s_wave[w];
  s_off[threadIdx.x] = off;
  __syncthreads();
  compact_group(bits, n_segs, g, s_off, s_stage, row_sel, out_sel);
}

__device__ __forceinline__ void compact_group(const uint64_t* __restrict__ bits, uint64_t n_segs, uint64_t group,
                                              const uint32_t* s_off, uint16_t (*s_stage)[kCompactStageRow],
                                              const uint32_t* __restrict__ row_sel, uint32_t* __restrict__ out_sel) {
  const uint64_t g0 = group * kGroupSegs;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
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
#if RPT_SEL_BALLOT_EXPAND
    // dense step (uniform): word by word, as unpermute_sel_kernel. The LDS staging below puts lane k's
    // survivors ~64p entries apart: at p = 1 every lane of a 2-B store hits one bank. Measured (C5
    // compact ms): p = 1.0 1.87 -> 0.76; at p = 0.5 the staging is faster (C5 10.66 vs 10.78 ms).
    if (total >= 8 * RPT_COMPACT_BALLOT_MIN) {
      uint32_t* dst = out_sel + s_off[b * 8];
      const uint32_t step_row = static_cast<uint32_t>(seg0 * kSegRows);
      uint32_t o = 0;
      for (int k = 0; k < 64; k++) {
        const uint64_t w = readlane64(word, k);
        if (w != 0) o += expand_word_sel(w, step_row + 64 * k, lane, row_sel, dst + o);  // uniform branch
      }
      continue;
    }
#endif
    uint32_t* dst = out_sel + s_off[b * 8];
    const uint32_t step_row = static_cast<uint32_t>(seg0 * kSegRows);
#if RPT_COMPACT_V16
    // entry j of the region is staged at buf[a + j], a = the destination's 4-B offset within its 16-B unit, so
    // staging unit u (buf[4u .. 4u+3], one 8-B LDS read) maps onto the aligned 16-B destination unit u
    const uint32_t a = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(dst) >> 2) & 3u;
    uint32_t p = incl - pc + a;
#else
    uint32_t p = incl - pc;
#endif
    while (word) {
      buf[p++] = static_cast<uint16_t>(lane * 64 + __builtin_ctzll(word));
      word &= word - 1;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#if RPT_COMPACT_V16
    uint32_t* base = dst - a;  // 16-B aligned
    const uint32_t end = a + total, n_units = (end + 3) >> 2;
    for (uint32_t u = lane; u < n_units; u += 64) {
      const uint64_t v4 = *reinterpret_cast<const uint64_t*>(buf + 4 * u);
      uint32_t r[4];
#pragma unroll
      for (int e = 0; e < 4; e++) {
        r[e] = step_row + static_cast<uint32_t>((v4 >> (16 * e)) & 0xffffu);
        if (row_sel && 4 * u + e >= a && 4 * u + e < end) r[e] = row_sel[r[e]];
      }
      if (4 * u >= a && 4 * u + 4 <= end) {
        *reinterpret_cast<u32x4*>(base + 4 * u) = u32x4{r[0], r[1], r[2], r[3]};
      } else {
#pragma unroll
        for (int e = 0; e < 4; e++)
          if (4 * u + e >= a && 4 * u + e < end) base[4 * u + e] = r[e];
      }
    }
#else
    for (uint32_t q = lane; q < total; q += 64) {
      const uint32_t row = step_row + buf[q];
      dst[q] = row_sel ? row_sel[row] : row;
    }
#endif
    __builtin_amdgcn_wave_barrier();
  }
}
}  // namespace rpt
