mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for x in 0 1; do
RPT_SLICE_XCD=$x timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_x$x.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_x$x.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('xcd',$x, d['value'], d['ms_per_step'], {k:round(v,3) for k,v in d['kernels_ms'].items()})"
done
