#!/usr/bin/env bash
# r04: the partition's rank-in-pass-1 form (RPT_PART_RANK1, int32 keys) -- parity of the variant, then a
# same-box alternating A/B against the claim-atomic form:
#   bash tools/build_variants.sh "rk0:-DRPT_PART_RANK1=0" "rk1:-DRPT_PART_RANK1=1"
set -o pipefail
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
RPT_GPU_LIB=$V/librpt_gpu_rk1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread > gpurun_out/rk1_parity.txt 2>&1 || { tail -30 gpurun_out/rk1_parity.txt; exit 1; }
tail -1 gpurun_out/rk1_parity.txt
bash tools/ab_args.sh "--config C2 --key-type i32|--config C2" rk0 rk1 && bash tools/ab_args.sh "--config C2 --key-type i32" rk0 rk1
