#!/usr/bin/env bash
# Stall-analysis counters for one bench config (memory-level parallelism, TA/TD/TCP stalls, L2->EA queue
# levels), one rocprofv3 --pmc pass per block-compatible set, summarised per kernel by pmc_summary.py.
#   bash tools/pmc_deep.sh OUTDIR TAG [bench args...]     (on the GPU box, from the repo root)
set -u
OUT=$1; TAG=$2; shift 2
BENCH_ARGS="$* --steps 3 --warmup 1 --no-cpu-baseline"
export TMPDIR=/tmp
mkdir -p "$OUT/pmc"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- python3 bench.py $BENCH_ARGS > "$OUT/trace.log" 2>&1 || { echo "trace pass failed"; exit 1; }
i=0
for ctr in "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT" \
           "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum" \
           "TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" \
           "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_sum" \
           "TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$OUT/pmc/p$i" -o run -- python3 bench.py $BENCH_ARGS > "$OUT/pmc/p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -3 "$OUT/pmc/p$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT/pmc" "$OUT/trace/bench_kernel_stats.csv" "$OUT/deep_$TAG.json" "$TAG"
