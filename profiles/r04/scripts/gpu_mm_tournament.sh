#!/usr/bin/env bash
# r04: the build's key min/max over a full NULL-free segment by a tournament (RPT_MM_TOURNAMENT=1) instead of a
# guarded min and max per value (bucketed level-1 scatter of the build): parity of the variant, then a same-box
# A/B on C5's share (insert_ms is the second number of each line)
#   bash tools/build_variants.sh "mt0:-DRPT_MM_TOURNAMENT=0" "mt1:-DRPT_MM_TOURNAMENT=1"
set -o pipefail
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
RPT_GPU_LIB=$V/librpt_gpu_mt1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_minmax_composite.py tests/test_gpu_bucketed.py tests/test_gpu_parity.py -k "minmax or bucketed or full_size or insert" -x -q --timeout 300 --timeout-method thread > gpurun_out/mt1_parity.txt 2>&1 || { tail -30 gpurun_out/mt1_parity.txt; exit 1; }
tail -1 gpurun_out/mt1_parity.txt
bash tools/ab_c5.sh mt0 mt1 && bash tools/ab_c5.sh mt0 mt1
