#!/usr/bin/env bash
# What the driver runs at round end, on one GPU box: the whole -m gpu suite, smoke(), and the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 1; }
python3 -c "import json;d=json.loads([l for l in open('gpurun_out/bench_default.json') if l.startswith('{')][0]);print(d['metric'], '%.4g'%d['value'], 'ms', round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],3), 'cpu', '%.3g'%d['cpu_baseline']['value'])"
