mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit 1
for args in "" "--build-rows 1e8"; do
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline $args > gpurun_out/bench.log 2>&1 || exit 1
python3 -c "import json;d=json.loads([l for l in open('gpurun_out/bench.log') if l.startswith('{')][-1]);print('$args', round(d['value']/1e9,1), 'Gkeys/s', 'build', d['build'])"
done
