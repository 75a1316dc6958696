set -o pipefail
mkdir -p gpurun_out
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "insert or full_size or golden" > gpurun_out/parity_dd.txt 2>&1 || { tail -5 gpurun_out/parity_dd.txt; exit 1; }
tail -1 gpurun_out/parity_dd.txt
bash tools/ab_c5.sh dd0 dd1 || exit 1
for rep in 1 2; do for v in dd0 dd1; do
  RPT_GPU_LIB=$V/librpt_gpu_$v.so timeout -k 10 200 python bench.py --config C3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab_c3_${v}_$rep.json 2>/dev/null || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], 'C3', round(d['ms_per_step'],3), round(d['build']['insert_ms'],3))" gpurun_out/ab_c3_${v}_$rep.json $v
done; done
RPT_GPU_LIB=$V/librpt_gpu_dd1.so timeout -k 10 200 python tools/insert_duplicates.py > gpurun_out/insert_duplicates_dd1.jsonl 2>/dev/null
