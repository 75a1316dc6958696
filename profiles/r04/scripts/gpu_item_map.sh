#!/usr/bin/env bash
# r04: bucket_unpermute finding each item's bucket through a per-item LDS table instead of a binary search
# (RPT_BUCKET_ITEM_MAP): parity of the variant on the bucketed tests, then a same-box A/B on C5's share
#   bash tools/build_variants.sh "im0:-DRPT_BUCKET_ITEM_MAP=0" "im1:-DRPT_BUCKET_ITEM_MAP=1"
set -o pipefail
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
RPT_GPU_LIB=$V/librpt_gpu_im1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_bucketed.py tests/test_gpu_parity.py -k "bucketed or full_size or C5" -x -q --timeout 300 --timeout-method thread > gpurun_out/im1_parity.txt 2>&1 || { tail -30 gpurun_out/im1_parity.txt; exit 1; }
tail -1 gpurun_out/im1_parity.txt
bash tools/ab_c5.sh im0 im1 && bash tools/ab_c5.sh im0 im1
