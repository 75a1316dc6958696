#!/usr/bin/env bash
# Quick HBM-bytes check of the bench's kernels: a kernel trace plus one --pmc pass each for FETCH_SIZE
# and WRITE_SIZE, summarised by tools/pmc_summary.py (FETCH doubled per the gfx950 correction).
#   bash tools/pmc_bytes.sh OUTDIR [bench args...]     (RPT_GPU_LIB selects a variant)
set -u
OUT=$1; shift
ARGS=${*:---steps 3 --warmup 1 --no-cpu-baseline}
export TMPDIR=/tmp
mkdir -p "$OUT/pmc"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1 || { echo "trace failed"; exit 1; }
i=0
for ctr in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$OUT/pmc/p$i" -o run -- python3 bench.py $ARGS > "$OUT/pmc/p$i.log" 2>&1 || { echo "pmc $ctr failed"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT/pmc" "$OUT/trace/bench_kernel_stats.csv" "$OUT/pmc_summary.json" quick > /dev/null
python3 - "$OUT/pmc_summary.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["kernels"]
for k, v in sorted(d.items(), key=lambda kv: -kv[1]["avg_ms"])[:8]:
    print(f"{k[:40]:40s} {v['avg_ms']:.3f} ms  rd {v['hbm_read_bytes']/1e9:.2f} GB  wr {v['hbm_write_bytes']/1e9:.2f} GB  {v['hbm_GBps']:.0f} GB/s")
PY
