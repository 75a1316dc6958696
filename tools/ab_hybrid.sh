#!/usr/bin/env bash
# A/B of the hybrid LDS/L2 direct probe (RPT_LDS_HYBRID_MAX_LOG > 14: the first 128 KiB of a 256 KiB..1 MiB filter in
# LDS, the rest gathered from L2) against AUTO (partitioned) and the plain gather, 1e9 int64 / int32 keys, 2 reps:
#   bash tools/ab_hybrid.sh BASE_VARIANT HYBRID_VARIANT
set -o pipefail
mkdir -p gpurun_out/ab
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
for rep in 1 2; do
for rows in 2e5 4e5 8e5; do
for kt in i64 i32; do
for run in "$1:auto" "$1:gather" "$2:lds"; do
  v=${run%%:*}; st=${run##*:}
  tag=hyb_${v}_${st}_${rows}_${kt}.$rep
  RPT_GPU_LIB=$V/librpt_gpu_$v.so timeout -k 10 200 python bench.py --build-rows $rows --filter-rows $rows --strategy $st --key-type $kt \
    --steps 10 --warmup 2 --no-cpu-baseline --no-stream-calibration > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "bench $tag failed"; tail -5 gpurun_out/ab/$tag.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], round(d['ms_per_step'],4), d['config']['probe_strategy'], d['config']['filter_bytes'], d['config']['pass_fraction'], {k[:22]: round(x,4) for k,x in list(d['kernels_ms'].items())[:3]})" gpurun_out/ab/$tag.json "$v $st $rows $kt"
done; done; done; done
