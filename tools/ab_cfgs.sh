#!/usr/bin/env bash
# A/B of librpt_gpu.so variants (tools/build_variants.sh) on bench configs, alternating, 2 reps:
#   AB_CFGS="C2 C3" bash tools/ab_cfgs.sh VARIANT...      (default configs: C2 C3)
set -o pipefail
mkdir -p gpurun_out
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
for rep in 1 2; do
for cfg in ${AB_CFGS:-C2 C3}; do
for v in "$@"; do
  RPT_GPU_LIB=$V/librpt_gpu_$v.so timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_${v}_${cfg}_$rep.json 2> gpurun_out/ab_${v}_${cfg}_$rep.err || { echo "bench $v $cfg failed"; tail -5 gpurun_out/ab_${v}_${cfg}_$rep.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],3), round(d['build']['insert_ms'],3), {k[:18]: round(x,3) for k,x in list(d['kernels_ms'].items())[:5]})" gpurun_out/ab_${v}_${cfg}_$rep.json $v "$cfg"
done; done; done
