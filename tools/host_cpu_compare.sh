#!/bin/bash
# The CPU restatement (bench.py's cpu_baseline leg: oracle/ C++ port, 2048-row vectors, hash included) at the
# thread counts tools/host_bench --host-path uses, for int64 and int32 keys against C2's filter: the host-side
# alternative each host-resident GPU rate is compared with. One JSON line per run.
set -e
cd "$(dirname "$0")/.."
for kt in i64 i32; do
  for t in 1 2 4 8 16; do
    timeout -k 5 120 python3 -u bench.py --cpu-baseline-only --config C2 --key-type "$kt" --cpu-threads "$t" --cpu-sample 1e8
  done
done
