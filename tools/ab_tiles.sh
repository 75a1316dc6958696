#!/usr/bin/env bash
# A/B of the 16 Ki- and 32 Ki-row partition tiles (tools/build_variants.sh t16 / t32): the GPU test
# suite against the t32 library, then C2 / C3 / C5-share bench lines for both, alternating.
set -o pipefail
mkdir -p gpurun_out
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
RPT_GPU_LIB=$V/librpt_gpu_t32.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_t32.log 2>&1 || { echo "t32 tests failed"; tail -30 gpurun_out/gpu_tests_t32.log; exit 1; }
tail -1 gpurun_out/gpu_tests_t32.log
for rep in 1 2; do
for cfg in "--build-rows 1e7" "--build-rows 1e8" "--build-rows 1e9 --filter-rows 8e9"; do
for v in t16 t32; do
  tag=$(echo "$cfg" | tr -d ' -')
  RPT_GPU_LIB=$V/librpt_gpu_$v.so timeout -k 10 200 python bench.py $cfg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_${v}_${tag}_$rep.json 2> gpurun_out/ab_${v}_${tag}_$rep.err || { echo "bench $v $cfg failed"; tail -5 gpurun_out/ab_${v}_${tag}_$rep.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],3), d['build']['insert_ms'], {k[:14]: round(x,3) for k,x in list(d['kernels_ms'].items())[:6]})" gpurun_out/ab_${v}_${tag}_$rep.json $v "$tag"
done; done; done
