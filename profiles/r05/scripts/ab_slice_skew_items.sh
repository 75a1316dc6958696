# Skew-aware slice probe work items (RPT_SLICE_SKEW_MULT): parity, uniform C2 / C3 A/B against the items off, skew sweep
set -o pipefail
mkdir -p gpurun_out
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/parity_skew.txt 2>&1 || { tail -15 gpurun_out/parity_skew.txt; exit 1; }
tail -1 gpurun_out/parity_skew.txt
for rep in 1 2 3; do for v in sk1 sk8; do for c in C2 C3; do
  RPT_GPU_LIB=$V/librpt_gpu_$v.so timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_sk_${v}_${c}_$rep.json 2>/dev/null || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],3), round(d['kernels_ms'].get('slice_probe_kernel',0),4), round(d['kernels_ms'].get('runs_transpose_kernel',0),4))" gpurun_out/ab_sk_${v}_${c}_$rep.json $v $c
done; done; done
RPT_GPU_LIB=$V/librpt_gpu_sk8.so timeout -k 10 300 python tools/probe_skew.py > gpurun_out/probe_skew_sk8.jsonl 2>/dev/null
