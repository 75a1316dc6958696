#!/usr/bin/env bash
# Multi-workgroup fused small probe: parity tests of the small paths, then latency one vs several workgroups
# (synchronized calls, keys in device and pinned host memory) and the kernels' durations under rocprofv3.
set -o pipefail
mkdir -p gpurun_out/small_mw
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chain.py tests/test_gpu_deferred_clear.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/small_mw/tests.log 2>&1 || { tail -30 gpurun_out/small_mw/tests.log; exit 1; }
tail -1 gpurun_out/small_mw/tests.log
timeout -k 10 200 python -u tools/small_probe_bench.py > gpurun_out/small_mw/latency.jsonl 2>&1 || { tail -20 gpurun_out/small_mw/latency.jsonl; exit 1; }
cat gpurun_out/small_mw/latency.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/small_mw/prof -o run -- python3 tools/small_probe_bench.py 16384 > gpurun_out/small_mw/prof.log 2>&1 || { tail -20 gpurun_out/small_mw/prof.log; exit 1; }
find gpurun_out/small_mw/prof -name '*kernel_stats.csv' -exec grep -h "probe_small\|Name" {} \;
