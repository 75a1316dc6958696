#!/usr/bin/env bash
# small-probe kernel durations with synchronized vs queued calls (rocprofv3 kernel trace, database output)
set -o pipefail
mkdir -p gpurun_out/small_mw2
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/small_mw2/prof -o run -- python3 tools/small_probe_bench.py ${SIZES:-16384} > gpurun_out/small_mw2/latency.jsonl 2>&1 || { tail -20 gpurun_out/small_mw2/latency.jsonl; exit 1; }
grep '^{' gpurun_out/small_mw2/latency.jsonl
