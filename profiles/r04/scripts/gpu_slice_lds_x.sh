#!/usr/bin/env bash
# r04 sensitivity of the slice probe to its random LDS reads: variants from profiles/r04/scripts/slice_lds_x.patch
#   bash tools/build_variants.sh "sl0:" "sl1:-DRPT_EXP_SLICE_LDS_X=1" "sl2:-DRPT_EXP_SLICE_LDS_X=2" "sl3:-DRPT_EXP_SLICE_LDS_X=3"
# sl1: one more random 8-B filter-word read per record, sl2: one more random mask-table read, sl3: both
# (masked by a run-time zero: results unchanged; 126 VGPRs, no spills, against 123).
set -o pipefail
bash tools/ab_args.sh "--config C2" sl0 sl1 sl2 sl3 && bash tools/ab_c5.sh sl0 sl3
