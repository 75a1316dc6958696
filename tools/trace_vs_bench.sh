#!/usr/bin/env bash
# Does the kernel tracer change kernel durations? The default bench untraced, then the SAME command under
# rocprofv3 --kernel-trace --stats (its bench line and its stats come from one process), then untraced again.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/tvb}; mkdir -p "$OUT"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_a.json" 2> "$OUT/bench_a.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- python3 bench.py --no-cpu-baseline > "$OUT/bench_traced.json" 2> "$OUT/bench_traced.err" || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_b.json" 2> "$OUT/bench_b.err" || exit 1
for f in bench_a bench_traced bench_b; do
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]);print(sys.argv[2], round(d['ms_per_step'],3), {k[:16]: round(x,3) for k,x in list(d['kernels_ms'].items())[:4]})" "$OUT/$f.json" $f
done
python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
  if 'rpt::' in r['Name']: print('stats', r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e6,4))
" "$OUT/trace/bench_kernel_stats.csv" | head -6
