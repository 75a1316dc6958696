mkdir -p gpurun_out; export TMPDIR=/tmp
for s in partitioned gather; do
timeout -k 10 300 python bench.py --build-rows 1e8 --strategy $s --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c3_$s.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_c3_$s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$s', round(d['value']/1e9,1), round(d['ms_per_step'],3), d['build'], {k:round(v,3) for k,v in d['kernels_ms'].items()})"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', round(d['value']/1e9,1), round(d['ms_per_step'],3), d['build'], {k:round(v,3) for k,v in d['kernels_ms'].items()})"
