// compaction.hpp — P2/P3: result bits -> ascending uint32 selection vector.
// Part of librpt_gpu.so: included by rpt_gpu.hip (one translation unit: kernels and their launches
// stay together without relocatable device code).
#pragma once

namespace rpt {

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
// Entries of each wave's staging buffer. 8 * RPT_COMPACT_BALLOT_MIN (3072, 6 KiB per wave) rather than a whole
// step's 4096 rows: 24 KiB of LDS per workgroup lets 6 workgroups share a CU instead of 4 (the kernel waits on
// its stores and LDS, so more waves hide more): C5 compaction 0.153-0.154 -> 0.130 ms at p = 0.1, 0.468 ->
// 0.426-0.430 ms at p = 0.5 (profiles/r05/ab_compact_stage.txt)
#ifndef RPT_COMPACT_STAGE
#define RPT_COMPACT_STAGE (RPT_SEL_BALLOT_EXPAND ? 8 * RPT_COMPACT_BALLOT_MIN : 8 * 512)
#endif
constexpr uint32_t kCompactStage = RPT_COMPACT_STAGE;
static_assert(kCompactStage == 8 * kSegRows || (RPT_SEL_BALLOT_EXPAND && kCompactStage >= 8 * RPT_COMPACT_BALLOT_MIN),
              "the LDS staging must hold every sparse step's survivors");
__global__ __launch_bounds__(kBlockThreads) void compact_kernel(const uint64_t* __restrict__ bits,
                                                               const uint32_t* __restrict__ seg_counts, uint64_t n_segs,
                                                               const uint32_t* __restrict__ group_offs,
                                                               const uint32_t* __restrict__ row_sel,
                                                               uint32_t* __restrict__ out_sel) {
  __shared__ uint32_t s_off[kGroupSegs];
  __shared__ uint32_t s_wave[kWavesPerBlock];
  // one 4096-row step's survivors per wave (row offsets); a step only stages when it has fewer than
  // 8 * RPT_COMPACT_BALLOT_MIN survivors (denser steps expand word by word), so that many entries suffice
  __shared__ uint16_t s_stage[kWavesPerBlock][kCompactStage];
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
}  // namespace rpt
