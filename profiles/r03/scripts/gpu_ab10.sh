#!/usr/bin/env bash
# r03: 8 Ki-row level-1 tiles (two scatter workgroups per CU, 78 KiB of LDS) vs 16 Ki, on the C5 share, with the
# whole-8-B-hash LDS sort; the bucketed tests on the 8 Ki variant first.
set -o pipefail
mkdir -p gpurun_out
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
RPT_GPU_LIB=$V/librpt_gpu_t8k.so timeout -k 10 600 python -u -m pytest tests/test_gpu_bucketed.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ab10.txt 2>&1 || { tail -40 gpurun_out/t_ab10.txt; exit 1; }
tail -1 gpurun_out/t_ab10.txt
bash tools/ab_c5.sh base t8k
