#!/usr/bin/env bash
# r04: the C5 bucket scatter's row map stored as one 2V-byte store per lane (RPT_SCATTER_POS_PACK=1; 2 = non-temporal)
# instead of V strided u16 stores: parity of the variants on the bucketed tests, then a same-box A/B on C5's share
#   bash tools/build_variants.sh "pp0:-DRPT_SCATTER_POS_PACK=0" "pp1:-DRPT_SCATTER_POS_PACK=1" "pp2:-DRPT_SCATTER_POS_PACK=2"
set -o pipefail
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
for v in pp1 pp2; do
  RPT_GPU_LIB=$V/librpt_gpu_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_bucketed.py tests/test_gpu_parity.py -k "bucketed or full_size or C5" -x -q --timeout 300 --timeout-method thread > gpurun_out/${v}_parity.txt 2>&1 || { tail -30 gpurun_out/${v}_parity.txt; exit 1; }
  tail -1 gpurun_out/${v}_parity.txt
done
bash tools/ab_c5.sh pp0 pp1 pp2 && bash tools/ab_c5.sh pp0 pp1 pp2
