mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --build-rows 1e9 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_big.log 2>&1 || { tail -5 gpurun_out/bench_big.log; exit 1; }
grep '^{' gpurun_out/bench_big.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('build 1e9', d['config'].get('probe_strategy'), round(d['value']/1e9,1), round(d['ms_per_step'],3), d['build'], {k:round(v,3) for k,v in d['kernels_ms'].items()})"
