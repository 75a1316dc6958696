# GPU check after a change: the whole -m gpu suite, then short bench lines for the given configs.
#   bash tools/gpu_check.sh TAG [CONFIG...]
set -o pipefail
mkdir -p gpurun_out
tag=$1; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/gpu_tests_$tag.txt 2>&1 || { tail -30 gpurun_out/gpu_tests_$tag.txt; exit 1; }
tail -1 gpurun_out/gpu_tests_$tag.txt
for cfg in "$@"; do
  timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_${tag}_$cfg.json 2> gpurun_out/bench_${tag}_$cfg.err || { tail -5 gpurun_out/bench_${tag}_$cfg.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], round(d['ms_per_step'],3), 'build', round(d['build']['insert_ms'],3), {k[:22]: round(x,3) for k,x in list(d['kernels_ms'].items())[:6]})" gpurun_out/bench_${tag}_$cfg.json $cfg
done
