#!/usr/bin/env bash
# One GPU-box pass that produces the round's evidence in one go: the GPU tests, the rocprofv3 kernel
# trace + PMC passes of the default bench (tools/profile_round.sh), the PMC summary installed as
# profiles/pmc_latest.json, then the default bench line (with the CPU baseline) run UNDER
# rocprofv3 --kernel-trace --stats, so the bench line and the kernel statistics committed beside it come
# from one process (boxes, and one box over minutes, differ by up to ~10 % in HBM rate).
#   bash tools/round_profile_and_bench.sh TAG      (outputs under gpurun_out/)
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 ||
  { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash tools/profile_round.sh gpurun_out/profile "$TAG" || exit 1
cp gpurun_out/profile/pmc_summary.json profiles/pmc_latest.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/benchtrace -o bench -- python3 bench.py \
  > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail gpurun_out/bench.err; exit 1; }
grep '^{' gpurun_out/bench.json
