#!/usr/bin/env bash
# r04 sensitivity of the C5 bucket scatter to its LDS bank conflicts: variants built by
#   bash tools/build_variants.sh "lx0:" "lx1:-DRPT_EXP_SCATTER_LDS_X=1" "lx2:-DRPT_EXP_SCATTER_LDS_X=2" "lx3:-DRPT_EXP_SCATTER_LDS_X=3"
# lx1 doubles the rank atomics' LDS work (a second no-return atomic per row on a copy of the counters),
# lx2 writes every row's 8-B sort slot twice, lx3 both (results unchanged). Then one PMC pass of the LDS
# counters for lx0 and lx3.
set -o pipefail
bash tools/ab_c5.sh lx0 lx1 lx2 lx3 && bash tools/ab_c5.sh lx0 lx1 lx2 lx3 || exit 1
export TMPDIR=/tmp
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
for v in lx0 lx3; do
  RPT_GPU_LIB=$V/librpt_gpu_$v.so timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES \
    --kernel-trace --output-format csv -d gpurun_out/ldsx/$v -o run -- python3 bench.py --build-rows 1e9 --filter-rows 8e9 --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/ldsx_$v.log 2>&1 || { echo "pmc $v failed"; tail -3 gpurun_out/ldsx_$v.log; exit 1; }
done
echo done
