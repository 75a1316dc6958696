#!/usr/bin/env bash
# A/B of librpt_gpu.so variants on arbitrary bench argument sets, alternating, 2 reps:
#   bash tools/ab_args.sh "ARGS1|ARGS2|..." VARIANT...
set -o pipefail
mkdir -p gpurun_out
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
IFS='|' read -ra SETS <<< "$1"; shift
for rep in 1 2; do
for args in "${SETS[@]}"; do
for v in "$@"; do
  tag=$(echo "$args" | tr -c 'a-zA-Z0-9' '_')
  RPT_GPU_LIB=$V/librpt_gpu_$v.so timeout -k 10 200 python bench.py $args --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/aba_${v}_${tag}_$rep.json 2> gpurun_out/aba_${v}_${tag}_$rep.err || { echo "bench $v $args failed"; tail -5 gpurun_out/aba_${v}_${tag}_$rep.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], '|', sys.argv[3], round(d['ms_per_step'],3), round(d['build']['insert_ms'],3), {k[:18]: round(x,3) for k,x in list(d['kernels_ms'].items())[:5]})" gpurun_out/aba_${v}_${tag}_$rep.json $v "$args"
done; done; done
