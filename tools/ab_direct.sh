#!/usr/bin/env bash
# A/B of direct-probe variants (tools/build_variants.sh) on the JOB-dimension filter (128 KiB, whole filter in LDS)
# and a 256 KiB gather, int64 and int32 keys, alternating, 3 reps:  bash tools/ab_direct.sh VARIANT...
set -o pipefail
mkdir -p gpurun_out/ab
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
for rep in 1 2 3; do
for args in "--config JOBDIM" "--config JOBDIM --key-type i32" "--build-rows 2e5 --filter-rows 2e5 --strategy gather"; do
for v in "$@"; do
  tag=$(echo "$v $args" | tr -c 'A-Za-z0-9\n' _)
  RPT_GPU_LIB=$V/librpt_gpu_$v.so timeout -k 10 200 python bench.py $args --steps 10 --warmup 2 --no-cpu-baseline --no-stream-calibration > gpurun_out/ab/$tag.$rep.json 2> gpurun_out/ab/$tag.$rep.err || { echo "bench $v $args failed"; tail -5 gpurun_out/ab/$tag.$rep.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],4), d['config']['pass_fraction'], {k[:22]: round(x,4) for k,x in list(d['kernels_ms'].items())[:3]})" gpurun_out/ab/$tag.$rep.json $v "$args"
done; done; done
