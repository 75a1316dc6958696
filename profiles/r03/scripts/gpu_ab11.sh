#!/usr/bin/env bash
# r03: the level-1 error path made conservative (probe passes every row, insert sets every bit): the bucketed
# tests (with the forced-error test of the test build), then a C5-share A/B against HEAD's build.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bucketed.py tests/test_gpu_bucketed_batches.py tests/test_abi.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ab11.txt 2>&1 || { tail -40 gpurun_out/t_ab11.txt; exit 1; }
tail -1 gpurun_out/t_ab11.txt
bash tools/ab_c5.sh base cons
