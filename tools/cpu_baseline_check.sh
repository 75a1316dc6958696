#!/bin/bash
# The single-filter CPU restatement two ways on the same host in one call (bench.py's cpu_baseline leg, probe_mt,
# at two sample sizes; the chain restatement with one filter), interleaved, 16 and 8 threads: whether the two
# agree and how much the sample size matters. One JSON line per run.
set -e
cd "$(dirname "$0")/.."
for rep in 1 2; do
  for t in 16 8; do
    for s in 100000000 33554432; do
      timeout -k 5 180 python3 -u bench.py --cpu-baseline-only --config C2 --cpu-threads "$t" --cpu-sample "$s"
    done
    timeout -k 5 180 python3 -u bench.py --cpu-baseline-only --config C2 --cpu-chain 1 --cpu-threads "$t" --cpu-sample 33554432
  done
done
