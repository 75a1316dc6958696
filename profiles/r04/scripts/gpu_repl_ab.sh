#!/usr/bin/env bash
# r04: the partition's replicated slice counters (RPT_PART_REPL) -- parity of the variant, then a
# same-box alternating A/B against single counters:
#   bash tools/build_variants.sh "rp0:-DRPT_PART_REPL=0" "rp16:-DRPT_PART_REPL=16"
set -o pipefail
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
RPT_GPU_LIB=$V/librpt_gpu_rp16.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_minmax_composite.py tests/test_gpu_chain.py tests/test_gpu_deferred_clear.py -x -q --timeout 300 --timeout-method thread > gpurun_out/rp16_parity.txt 2>&1 || { tail -30 gpurun_out/rp16_parity.txt; exit 1; }
tail -1 gpurun_out/rp16_parity.txt
bash tools/ab_args.sh "--config C2 --key-type i32|--config C2" rp0 rp16 && bash tools/ab_args.sh "--config C2 --key-type i32" rp0 rp16
