#!/usr/bin/env bash
# One GPU-box pass: the GPU test suite, the host-mirror bench, then an A/B of librpt_gpu.so variants
# (built by tools/build_variants.sh) on the default bench, alternating. Every GPU step has its own
# time limit; the first failure ends the pass.
#   bash tools/gpu_check.sh [--no-tests] [variant ...]
set -o pipefail
mkdir -p gpurun_out
TESTS=1
if [ "${1:-}" = "--no-tests" ]; then TESTS=0; shift; fi
if [ $TESTS = 1 ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
  timeout -k 10 300 ./tools/host_bench/build/host_bench > gpurun_out/host_bench.jsonl 2> gpurun_out/host_bench.err || { echo "host bench failed"; cat gpurun_out/host_bench.err; exit 1; }
  cat gpurun_out/host_bench.jsonl
fi
VARIANTS=("$@")
for rep in 1 2; do
  for v in "${VARIANTS[@]}"; do
    RPT_GPU_LIB=$PWD/duckdb-robust-predicate-transfer_amd/build/variants/librpt_gpu_$v.so timeout -k 10 300 \
      python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_${v}_$rep.json 2> gpurun_out/ab_${v}_$rep.err ||
      { echo "bench $v failed"; tail gpurun_out/ab_${v}_$rep.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], round(d['ms_per_step'],4), {k[:28]: round(x,4) for k,x in list(d['kernels_ms'].items())[:5]})" gpurun_out/ab_${v}_$rep.json $v
  done
done
