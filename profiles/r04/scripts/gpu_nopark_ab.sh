#!/usr/bin/env bash
# r04: the partition's records-in-registers form (no LDS park) (RPT_PART_NOPARK, int32 keys) -- parity of the variant, then a
# same-box alternating A/B against the parked form:
#   bash tools/build_variants.sh "np0:-DRPT_PART_NOPARK=0" "np1:-DRPT_PART_NOPARK=1"
set -o pipefail
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
RPT_GPU_LIB=$V/librpt_gpu_np1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread > gpurun_out/np1_parity.txt 2>&1 || { tail -30 gpurun_out/np1_parity.txt; exit 1; }
tail -1 gpurun_out/np1_parity.txt
bash tools/ab_args.sh "--config C2 --key-type i32|--config C2" np0 np1 && bash tools/ab_args.sh "--config C2 --key-type i32" np0 np1
