set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bucketed.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_buck.txt 2>&1 || { tail -40 gpurun_out/t_buck.txt; exit 1; }
tail -2 gpurun_out/t_buck.txt
timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_C5.json 2> gpurun_out/bench_C5.err || { tail -5 gpurun_out/bench_C5.err; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(round(d['ms_per_step'],3), 'build', round(d['build']['insert_ms'],3), {k[:24]: round(x,3) for k,x in list(d['kernels_ms'].items())[:9]})" gpurun_out/bench_C5.json
