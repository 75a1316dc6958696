mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for cfg in "--filter-rows 8e9 --build-rows 1e9" "--build-rows 1e7"; do
timeout -k 10 400 python bench.py $cfg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_cfg.log 2>&1 || { tail -5 gpurun_out/bench_cfg.log; exit 1; }
grep '^{' gpurun_out/bench_cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'][:24], d['config'].get('probe_strategy'), round(d['value']/1e9,1), round(d['ms_per_step'],3), round(d['build']['insert_ms'],3), {k:round(v,3) for k,v in d['kernels_ms'].items()})"
done
