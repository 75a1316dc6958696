#!/usr/bin/env bash
# A/B of librpt_gpu.so variants on one rank's share of C5 (8 GiB filter, 1e9 build + 1e9 probe keys):
#   bash tools/ab_c5.sh VARIANT...
set -o pipefail
mkdir -p gpurun_out
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
for rep in 1 2; do
for v in "$@"; do
  RPT_GPU_LIB=$V/librpt_gpu_$v.so timeout -k 10 300 python bench.py --build-rows 1e9 --filter-rows 8e9 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab_c5_${v}_$rep.json 2> gpurun_out/ab_c5_${v}_$rep.err || { echo "bench $v failed"; tail -5 gpurun_out/ab_c5_${v}_$rep.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], 'C5share', round(d['ms_per_step'],3), round(d['build']['insert_ms'],3), {k[:14]: round(x,3) for k,x in list(d['kernels_ms'].items())[:6]})" gpurun_out/ab_c5_${v}_$rep.json $v
done; done
