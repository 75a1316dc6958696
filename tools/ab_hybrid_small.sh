#!/usr/bin/env bash
# The hybrid LDS/L2 probe against the gather at small batches (its 128 KiB LDS staging per workgroup is a fixed
# cost): 256 / 512 KiB filters, 2^16 .. 2^22 probe rows, int64, 200 timed steps each, alternating, 2 reps.
set -o pipefail
mkdir -p gpurun_out/ab
for rep in 1 2; do
for rows in 2e5 4e5; do
for n in 65536 262144 1048576 4194304; do
for st in gather lds; do
  tag=hs_${rows}_${n}_${st}.$rep
  timeout -k 10 200 python bench.py --build-rows $rows --filter-rows $rows --probe-rows $n --strategy $st --steps 200 \
    --warmup 20 --no-cpu-baseline --no-stream-calibration > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "bench $tag failed"; tail -5 gpurun_out/ab/$tag.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], round(d['ms_per_step']*1000,2), 'us/step', round(d['probe_total']['avg_ms']*1000,2), 'us device', {k[:24]: round(x*1000,2) for k,x in list(d['kernels_ms'].items())[:2]})" gpurun_out/ab/$tag.json "$rows $n $st"
done; done; done; done
