#!/bin/bash
# The CPU restatement of USE_BF's filter loop (bench.py --cpu-baseline-only --cpu-chain K: oracle/ C++ port, 2048-row
# vectors, filter f over the survivors of filters 0..f-1, hash included) for the shape tools/host_bench --chain
# measures on the GPU (2^25 rows; BIGINT 10 % hits, INTEGER 50 %, BIGINT 50 %), at 1 / 8 / 16 threads. One JSON
# line per run.
set -e
cd "$(dirname "$0")/.."
for k in 1 2 3; do
  for t in 1 8 16; do
    timeout -k 5 180 python3 -u bench.py --cpu-baseline-only --config C2 --cpu-chain "$k" --cpu-threads "$t" --cpu-sample 33554432
  done
done
