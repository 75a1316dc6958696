#!/usr/bin/env bash
# Profile one bench config on the GPU box: kernel-trace stats + one rocprofv3 --pmc pass per counter
# set (never combined with other trace domains), then the per-kernel summary, installed as
# profiles/pmc/<CONFIG>.json (the file bench.py reads for that config's `traffic` fields).
# Usage (on the box, from the repo root):
#   bash tools/profile_round.sh OUTDIR CONFIG ROUND [bench args...]
#   e.g. bash tools/profile_round.sh gpurun_out/prof_c3 C3 r02 --config C3
set -u
OUT=$1; CFG=$2; TAG=$3; shift 3
BENCH_ARGS="$* --steps 5 --warmup 1 --no-cpu-baseline"
export TMPDIR=/tmp
mkdir -p "$OUT/pmc" profiles/pmc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- python3 bench.py $BENCH_ARGS > "$OUT/bench_trace.log" 2>&1 || { echo "trace pass failed"; exit 1; }
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$OUT/pmc/p$i" -o run -- python3 bench.py $BENCH_ARGS > "$OUT/pmc/p$i.log" 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT/pmc" "$OUT/trace/bench_kernel_stats.csv" "profiles/pmc/$CFG.json" "$TAG"
cp "profiles/pmc/$CFG.json" "$OUT/pmc_summary.json"  # gpurun merges back only gpurun_out/
