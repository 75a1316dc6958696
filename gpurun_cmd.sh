mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1; echo "prof rc=$?"
  python - <<'PY'
import csv, json
for r in csv.DictReader(open('gpurun_out/prof/bench_kernel_stats.csv')):
    print(f"{r['Name'][:50]:50s} calls={r['Calls']:>3} avg_ms={float(r['AverageNs'])/1e6:8.3f}")
d = json.loads(open('gpurun_out/bench_prof.log').read().strip().splitlines()[-1])
print("value Gkeys/s", d["value"]/1e9, "p1_ms", d["roofline"]["avg_launch_ms"], "probe_ms", d["probe_total"]["avg_ms"])
PY
fi
