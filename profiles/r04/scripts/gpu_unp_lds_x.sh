#!/usr/bin/env bash
# r04 sensitivity of unpermute_sel to its random pass-bit LDS reads (patch unp_lds_x.patch):
#   bash tools/build_variants.sh "ux0:" "ux1:-DRPT_EXP_UNP_LDS_X=1"
# ux1 reads every row's pass-bit word a second time (masked by a run-time zero: results unchanged).
set -o pipefail
bash tools/ab_args.sh "--config C2|--config C2 --p 0.5" ux0 ux1
