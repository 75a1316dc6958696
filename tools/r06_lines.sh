#!/usr/bin/env bash
# r06 evidence on one GPU box: the CPU baseline's placement x prefetch-distance sweep, then per
# config the rocprofv3 kernel trace + PMC passes (profiles/pmc/<config>.json) and the bench line run under
# rocprofv3 --kernel-trace --stats (tools/round_profile_and_bench.sh), then optionally the C5 section at full size
# on one rank (per-rank device memory with the on-device merge check).
#   bash tools/r06_lines.sh "C2 C3" [c5]
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06
CFGS=$1
if [ -n "${CPU_SWEEP:-}" ]; then
  timeout -k 10 300 python3 bench.py --cpu-baseline-only --cpu-threads 16 --cpu-lag-sweep 24,2048 --cpu-pin-sweep 0,1,2 \
    --cpu-sweep-rounds 3 --cpu-sample 1e9 > gpurun_out/r06/cpu_pin_lag_16t.json || exit 1
fi
SKIP_TESTS=1 bash tools/round_profile_and_bench.sh r06 $CFGS > gpurun_out/r06/lines_$(echo $CFGS | tr ' ' _).log 2>&1 || { tail -30 gpurun_out/r06/lines_*.log; exit 1; }
if [ "${2:-}" = c5 ]; then
  timeout -k 10 300 python3 bench.py --c5-merge --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r06/c5_section_n1_full.json 2> gpurun_out/r06/c5_section_n1_full.err || exit 1
fi
echo done
