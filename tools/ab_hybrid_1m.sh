#!/usr/bin/env bash
# 1 MiB filters (8e5 keys): the hybrid LDS/L2 probe (variant h17) against the gather AUTO runs below 2^25 rows,
# 2^21 .. 2^25 probe rows, int64 and int32, 100 timed steps, alternating, 2 reps.
set -o pipefail
mkdir -p gpurun_out/ab
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
for rep in 1 2; do
for kt in i64 i32; do
for n in 2097152 4194304 8388608 16777216 33554432; do
for st in gather lds; do
  tag=h1m_${kt}_${n}_${st}.$rep
  RPT_GPU_LIB=$V/librpt_gpu_h17.so timeout -k 10 200 python bench.py --build-rows 8e5 --filter-rows 8e5 --probe-rows $n --key-type $kt \
    --strategy $st --steps 100 --warmup 10 --no-cpu-baseline --no-stream-calibration > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "bench $tag failed"; tail -5 gpurun_out/ab/$tag.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], round(d['ms_per_step']*1000,1), 'us/step')" gpurun_out/ab/$tag.json "$kt $n $st"
done; done; done; done
