#!/usr/bin/env bash
# SURVEY §8d pass-fraction sweep: bench lines at p in {0.01, 0.1, 0.5, 1.0} per config.
#   bash tools/p_sweep.sh [CONFIG ...]      (default: C2 C3; outputs gpurun_out/psweep_<cfg>_<p>.json)
set -o pipefail
mkdir -p gpurun_out
for cfg in ${*:-C2 C3}; do
  for p in 0.01 0.1 0.5 1.0; do
    timeout -k 10 300 python bench.py --config $cfg --p $p --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/psweep_${cfg}_$p.json 2> gpurun_out/psweep_${cfg}_$p.err || { tail -5 gpurun_out/psweep_${cfg}_$p.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], 'p', sys.argv[3], 'ms', round(d['ms_per_step'],3), 'keys/s %.3g' % d['value'], 'pass', d['config']['pass_fraction'], {k[:22]: round(x,3) for k,x in list(d['kernels_ms'].items())[:4]})" gpurun_out/psweep_${cfg}_$p.json $cfg $p
  done
done
