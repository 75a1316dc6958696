#!/usr/bin/env bash
# r04: the records-in-registers partition for 32 Ki-row tiles (C3: 1024 slices, one workgroup per CU, 128-VGPR budget;
# 115 used, no spills): parity of the variant, then a same-box alternating A/B on C3 (int64 and int32 keys)
#   bash tools/build_variants.sh "tp1:-DRPT_PART_NOPARK=1" "tp3:-DRPT_PART_NOPARK=3"     (patch part_nopark_tm2.patch)
set -o pipefail
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
RPT_GPU_LIB=$V/librpt_gpu_tp3.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_minmax_composite.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tp3_parity.txt 2>&1 || { tail -30 gpurun_out/tp3_parity.txt; exit 1; }
tail -1 gpurun_out/tp3_parity.txt
bash tools/ab_args.sh "--config C3|--config C3 --key-type i32" tp1 tp3
