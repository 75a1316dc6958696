#!/usr/bin/env bash
# Copy one tools/round_profile_and_bench.sh run (merged back under gpurun_out/) into the tracked
# evidence: profiles/pmc/<CONFIG>.json (what bench.py reads for `traffic`), profiles/<ROUND>/bench_<CONFIG>.json
# and the kernel statistics of the same traced bench process, and the GPU test log.
#   bash tools/collect_evidence.sh ROUND CONFIG...
set -euo pipefail
R=$1; shift
mkdir -p profiles/pmc "profiles/$R"
for c in "$@"; do
  cp "gpurun_out/prof_$c/pmc_summary.json" "profiles/pmc/$c.json"
  grep '^{' "gpurun_out/bench_$c.json" > "profiles/$R/bench_$c.json"
  cp "gpurun_out/benchtrace_$c/bench_kernel_stats.csv" "profiles/$R/bench_${c}_kernel_stats.csv"
done
if [ -f gpurun_out/gpu_tests.log ]; then cp gpurun_out/gpu_tests.log "profiles/$R/gpu_tests.txt"; fi
