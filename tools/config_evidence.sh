#!/usr/bin/env bash
# Bench lines + kernel statistics (one traced process each) for the non-default configs:
# C3 (1e8-key build, 128 MiB filter, 1e9-key probe), one rank's share of C5 (8 GiB filter), C2 with
# int32 keys, and a JOB-sized 128 KiB filter (1e5 build keys: whole-filter LDS probe).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg
run() {
  local tag=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cfg/$tag -o bench -- python3 bench.py "$@" \
    > gpurun_out/cfg/$tag.json 2> gpurun_out/cfg/$tag.err || { echo "$tag failed"; tail gpurun_out/cfg/$tag.err; exit 1; }
  grep '^{' gpurun_out/cfg/$tag.json | cut -c1-200
}
run c3 --build-rows 1e8 --cpu-sample 2e8 || exit 1
run c5_share --build-rows 1e9 --filter-rows 8e9 --steps 10 --warmup 2 --cpu-sample 1e8 || exit 1
run c2_int32 --key-type i32 || exit 1
run job_dim_128k --build-rows 1e5 || exit 1
