#!/usr/bin/env bash
# A/B of library variants on the 256 KiB filter (hybrid LDS/L2 probe), int64 and int32, alternating, 3 reps:
#   bash tools/ab_hybrid_group.sh VARIANT...
set -o pipefail
mkdir -p gpurun_out/ab
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
for rep in 1 2 3; do
for kt in i64 i32; do
for v in "$@"; do
  tag=hg_${v}_${kt}.$rep
  RPT_GPU_LIB=$V/librpt_gpu_$v.so timeout -k 10 200 python bench.py --config JOBDIM256 --key-type $kt --steps 10 --warmup 2 \
    --no-cpu-baseline --no-stream-calibration > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "bench $tag failed"; tail -5 gpurun_out/ab/$tag.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], round(d['ms_per_step'],4), {k[:26]: round(x,4) for k,x in list(d['kernels_ms'].items())[:2]})" gpurun_out/ab/$tag.json "$v $kt"
done; done; done
