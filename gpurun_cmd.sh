mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
V=duckdb-robust-predicate-transfer_amd/build/variants
for x in base noscatter nocount; do
  if [ $x = base ]; then L=duckdb-robust-predicate-transfer_amd/build/librpt_gpu.so; else L=$V/librpt_gpu_$x.so; fi
  RPT_GPU_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$x.log 2>&1 || { echo "$x failed"; tail -5 gpurun_out/bench_$x.log; exit 1; }
  grep '^{' gpurun_out/bench_$x.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$x', round(d['value']/1e9,1), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['kernels_ms'].items()})"
done
