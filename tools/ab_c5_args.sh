#!/usr/bin/env bash
# A/B of librpt_gpu.so variants on one rank's share of C5 with extra bench args (e.g. --p 0.5), alternating, 2 reps:
#   bash tools/ab_c5_args.sh "EXTRA ARGS" VARIANT...
set -o pipefail
mkdir -p gpurun_out
X=$1; shift
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
tag=$(echo "$X" | tr -c 'a-zA-Z0-9' '_')
for rep in 1 2; do
for v in "$@"; do
  RPT_GPU_LIB=$V/librpt_gpu_$v.so timeout -k 10 300 python bench.py --build-rows 1e9 --filter-rows 8e9 --steps 5 --warmup 1 --no-cpu-baseline $X > gpurun_out/abx_${v}_${tag}_$rep.json 2> gpurun_out/abx_${v}_${tag}_$rep.err || { echo "bench $v failed"; tail -5 gpurun_out/abx_${v}_${tag}_$rep.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], sys.argv[3], 'C5share', round(d['ms_per_step'],3), {k[:14]: round(x,3) for k,x in list(d['kernels_ms'].items())[:7]})" gpurun_out/abx_${v}_${tag}_$rep.json $v "$X"
done; done
