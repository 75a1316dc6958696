/*
 * rpt_gpu_synth.h — device-side generators of the synthetic benchmark workload.
 * Bench/test support exported by librpt_gpu.so; not part of the PTBloomFilter seam.
 *
 *   build key i  = (int64) splitmix64(RPT_SYNTH_SEED_BUILD, i)
 *   probe row r  : u = splitmix64(RPT_SYNTH_SEED_PROBE_SEL, r)
 *                  (u % 1000) < p_permille ? build key ((u >> 20) % n_build)
 *                                          : (int64) splitmix64(RPT_SYNTH_SEED_PROBE_MISS, r)
 *   splitmix64(seed, i) = mix64(seed + (i + 1) * 0x9e3779b97f4a7c15)
 * The same streams are restated on the host by oracle/rpt_oracle.cpp for parity checks.
 */
#ifndef RPT_GPU_SYNTH_H
#define RPT_GPU_SYNTH_H

#include <stdint.h>

#include "rpt_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RPT_SYNTH_SEED_BUILD 0x5EED0001ULL
#define RPT_SYNTH_SEED_PROBE_SEL 0x5EED0002ULL
#define RPT_SYNTH_SEED_PROBE_MISS 0x5EED0003ULL

/* out[i] = build key (start + i), i < n (device pointer). */
int rpt_synth_build_keys(int64_t* out, uint64_t start, uint64_t n, rpt_stream_t stream);
/* out[i] = probe key of row (start + i), i < n (device pointer). */
int rpt_synth_probe_keys(int64_t* out, uint64_t n_build, uint32_t p_permille, uint64_t start, uint64_t n,
                         rpt_stream_t stream);

/* Stream calibration (bench.py reports the kernels' HBM fractions against what this box streams, beside the
 * 8 TB/s spec): read `bytes` bytes at `src` with 16-B non-temporal loads, 8 in flight per lane, over a grid of
 * 16 x 256-thread workgroups per CU (sink: one word per workgroup, rpt_stream_sink_words(device) words), or copy
 * them to `dst` (one 16-B unit per lane). The fastest of the variants tools/ubench/ubench_stream.hip times.
 * Device pointers, 16-B aligned, bytes a multiple of 16. Stream-ordered, no sync. */
uint64_t rpt_stream_sink_words(int device);
int rpt_stream_read(const void* src, uint64_t bytes, uint64_t* sink, rpt_stream_t stream);
int rpt_stream_copy(void* dst, const void* src, uint64_t bytes, rpt_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* RPT_GPU_SYNTH_H */
