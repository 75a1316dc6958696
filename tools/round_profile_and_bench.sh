#!/usr/bin/env bash
# One GPU-box pass that produces a round's evidence: the GPU tests, then per config the rocprofv3
# kernel trace + PMC passes (tools/profile_round.sh -> profiles/pmc/<config>.json), then the bench line
# (with the CPU baseline) run UNDER rocprofv3 --kernel-trace --stats, so the bench line and the kernel
# statistics committed beside it come from one process.
#   bash tools/round_profile_and_bench.sh ROUND [CONFIG ...]     (default configs: C2; outputs under gpurun_out/)
#   SKIP_TESTS=1 skips the GPU tests (a second call for more configs within gpurun's 20-minute limit)
set -o pipefail
TAG=${1:-r02}; shift || true
CFGS=${*:-C2}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 ||
    { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
for c in $CFGS; do
  case $c in
    *-i32) args="--config ${c%-i32} --key-type i32" ;;
    *) args="--config $c" ;;
  esac
  bash tools/profile_round.sh gpurun_out/prof_$c "$c" "$TAG" $args || exit 1
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/benchtrace_$c -o bench -- python3 bench.py $args \
    > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo "bench $c failed"; tail gpurun_out/bench_$c.err; exit 1; }
  grep '^{' gpurun_out/bench_$c.json
done
