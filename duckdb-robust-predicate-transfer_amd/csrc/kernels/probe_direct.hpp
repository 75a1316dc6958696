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
    bool pass[8];
#pragma unroll
    for (int j = 0; j < 8; j++) pass[j] = ok[j] && (w[j] & m[j]) == m[j];
    store_segment_bits<K, DENSE>(pass, lane, seg, out_bits, seg_counts);
  }
}
}  // namespace rpt
