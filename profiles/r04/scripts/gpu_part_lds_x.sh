#!/usr/bin/env bash
# r04 sensitivity of the C2 partition kernel to its LDS work (int64 and int32 keys): variants built by
#   bash tools/build_variants.sh "px0:" "px1:-DRPT_EXP_PART_LDS_X=1" "px2:-DRPT_EXP_PART_LDS_X=2" \
#     "px4:-DRPT_EXP_PART_LDS_X=4" "px7:-DRPT_EXP_PART_LDS_X=7"
# from profiles/r04/scripts/part_lds_x.patch: 1 = the pass-1 count atomic twice, 2 = the pass-2 claim atomic
# twice, 4 = the slice-sorted placement write twice, 7 = all three (results unchanged).
set -o pipefail
bash tools/ab_args.sh "--config C2|--config C2 --key-type i32" px0 px1 px2 px4 px7 || exit 1
export TMPDIR=/tmp
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
for v in px0 px7; do
  RPT_GPU_LIB=$V/librpt_gpu_$v.so timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES \
    --kernel-trace --output-format csv -d gpurun_out/partx/$v -o run -- python3 bench.py --config C2 --key-type i32 --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/partx_$v.log 2>&1 || { echo "pmc $v failed"; tail -3 gpurun_out/partx_$v.log; exit 1; }
done
echo done
