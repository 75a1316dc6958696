#!/usr/bin/env bash
# A/B of environment settings on one bench config, alternating, 2 reps:
#   bash tools/ab_env.sh "BENCH ARGS" "ENV1" "ENV2" ...     (ENV "-" = none)
set -o pipefail
mkdir -p gpurun_out
CFG=$1; shift
for rep in 1 2; do
for e in "$@"; do
  tag=$(echo "$e$CFG" | tr -c 'a-zA-Z0-9' '_')
  envs=(); [ "$e" != "-" ] && envs=($e)
  env "${envs[@]}" timeout -k 10 300 python bench.py $CFG --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/abe_${tag}_$rep.json 2> gpurun_out/abe_${tag}_$rep.err || { echo "bench $e failed"; tail -5 gpurun_out/abe_${tag}_$rep.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], '|', sys.argv[3], round(d['ms_per_step'],3), round(d['build']['insert_ms'],3), {k[:14]: round(x,3) for k,x in list(d['kernels_ms'].items())[:5]})" gpurun_out/abe_${tag}_$rep.json "$e" "$CFG"
done; done
