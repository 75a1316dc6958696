#!/usr/bin/env bash
# r04: the records-in-registers partition (RPT_PART_NOPARK) extended to hash keys and to the bucketed level 2's
# split hashes (RPT_PART_NOPARK=2): parity of the variant, then a same-box alternating A/B on C5's share
#   bash tools/build_variants.sh "nk1:-DRPT_PART_NOPARK=1" "nk2:-DRPT_PART_NOPARK=2"
set -o pipefail
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
RPT_GPU_LIB=$V/librpt_gpu_nk2.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_bucketed.py tests/test_gpu_bucketed_batches.py tests/test_gpu_minmax_composite.py tests/test_gpu_chain.py -x -q --timeout 300 --timeout-method thread > gpurun_out/nk2_parity.txt 2>&1 || { tail -30 gpurun_out/nk2_parity.txt; exit 1; }
tail -1 gpurun_out/nk2_parity.txt
bash tools/ab_c5.sh nk1 nk2 && bash tools/ab_c5.sh nk1 nk2
