#!/usr/bin/env bash
# r03: USE_BF's filter chain in one launch (rpt_bf_probe_chain): its GPU tests, the C++ host mirror test, the
# small-probe parity tests it shares a tail with, then the host bench (per-vector chain vs filter by filter)
# under the kernel tracer (kernel durations of the small probe and the chain kernel).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_host_mirror.py tests/test_gpu_parity.py tests/test_readme_join.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_chain.txt 2>&1 || { tail -40 gpurun_out/t_chain.txt; exit 1; }
tail -2 gpurun_out/t_chain.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hbtrace -o hb -- ./tools/host_bench/build/host_bench > gpurun_out/host_bench.jsonl 2> gpurun_out/host_bench.err || { tail -5 gpurun_out/host_bench.err; exit 1; }
grep -E "probe_small|probe_chain" gpurun_out/hbtrace/hb_kernel_stats.csv | cut -c1-60,180-260
grep -E "UseBF|\"LookupSel\"" gpurun_out/host_bench.jsonl
