# A/B of the slice probe's work-item count (RPT_SLICE_SPLIT_MULT) under probe-key skew and on uniform C2 / C3
set -o pipefail
mkdir -p gpurun_out
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
for v in m1 m4 m8; do
  RPT_GPU_LIB=$V/librpt_gpu_$v.so timeout -k 10 300 python tools/probe_skew.py > gpurun_out/probe_skew_$v.jsonl 2>/dev/null || exit 1
done
for rep in 1 2; do for v in m1 m4 m8; do for c in C2 C3; do
  RPT_GPU_LIB=$V/librpt_gpu_$v.so timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_sm_${v}_${c}_$rep.json 2>/dev/null || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],3), round(d['kernels_ms'].get('slice_probe_kernel',0),3))" gpurun_out/ab_sm_${v}_${c}_$rep.json $v $c
done; done; done
