#!/usr/bin/env bash
# r06: the GPU suite (timed), the CPU baseline's interleaved prefetch-lag sweep on the box's host (VERDICT r05
# item 6), and the C5 section at full size on one rank (per-rank device memory with the on-device merge check).
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=25 > gpurun_out/r06/gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r06/gpu_tests.txt; exit 1; }
tail -3 gpurun_out/r06/gpu_tests.txt
timeout -k 10 200 python3 bench.py --cpu-baseline-only --cpu-threads 16 --cpu-lag-sweep 24,128,2048 --cpu-sweep-rounds 4 --cpu-sample 1e9 > gpurun_out/r06/cpu_lag_interleaved_16t.json || exit 1
timeout -k 10 200 python3 bench.py --cpu-baseline-only --cpu-threads 1 --cpu-lag-sweep 24,2048 --cpu-sweep-rounds 2 --cpu-sample 2e8 > gpurun_out/r06/cpu_lag_interleaved_1t.json || exit 1
