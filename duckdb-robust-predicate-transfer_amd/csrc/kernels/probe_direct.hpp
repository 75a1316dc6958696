// probe_direct.hpp — P1: hash + filter gather (global or whole-filter LDS) -> result bits.
// Part of librpt_gpu.so: included by rpt_gpu.hip (one translation unit: kernels and their launches
// stay together without relocatable device code).
#pragma once

namespace rpt {

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
}  // namespace rpt
