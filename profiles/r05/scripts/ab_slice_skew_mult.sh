# RPT_SLICE_SKEW_MULT 8 / 16 / 32: skew sweep and uniform C2 / C3
set -o pipefail
mkdir -p gpurun_out
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
for v in sk8 sk16 sk32; do
  RPT_GPU_LIB=$V/librpt_gpu_$v.so timeout -k 10 300 python tools/probe_skew.py > gpurun_out/probe_skew_$v.jsonl 2>/dev/null || exit 1
done
for rep in 1 2; do for v in sk8 sk16 sk32; do for c in C2 C3; do
  RPT_GPU_LIB=$V/librpt_gpu_$v.so timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_skm_${v}_${c}_$rep.json 2>/dev/null || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],3), round(d['kernels_ms'].get('slice_probe_kernel',0),4))" gpurun_out/ab_skm_${v}_${c}_$rep.json $v $c
done; done; done
