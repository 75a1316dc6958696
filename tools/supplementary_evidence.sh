#!/usr/bin/env bash
# r06 supplementary evidence: stream-rate kernel variants, the CPU baseline's
# prefetch-distance sweep at 1 and 16 threads, and the JOB-dimension filter profiled (int64 + int32).
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06
timeout -k 10 120 tools/ubench/ubench_stream > gpurun_out/r06/ubench_stream.txt 2>&1 || exit 1
for t in 1 16; do for lag in 24 128 2048; do
  timeout -k 10 200 python3 bench.py --cpu-baseline-only --cpu-threads $t --cpu-lag $lag --cpu-sample 2e8 >> gpurun_out/r06/cpu_lag_sweep.jsonl || exit 1
done; done
SKIP_TESTS=1 bash tools/round_profile_and_bench.sh r06 JOBDIM JOBDIM-i32 > gpurun_out/r06/jobdim.log 2>&1 || { tail -20 gpurun_out/r06/jobdim.log; exit 1; }
tail -3 gpurun_out/r06/jobdim.log
