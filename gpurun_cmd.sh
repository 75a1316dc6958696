mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/profile
bash tools/profile_round.sh gpurun_out/profile r01 > gpurun_out/profile_round.log 2>&1 || { tail -5 gpurun_out/profile_round.log; exit 1; }
cp gpurun_out/profile/pmc_summary.json profiles/pmc_latest.json
timeout -k 10 300 python bench.py > gpurun_out/bench_final.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_final.log > gpurun_out/bench_final.json
python3 -c "import json; d=json.load(open('gpurun_out/bench_final.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d['cpu_baseline']['value'])"
