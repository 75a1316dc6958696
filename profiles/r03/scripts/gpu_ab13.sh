#!/usr/bin/env bash
# r03 measurement only: the slice probe with its pass-bit stores skipped (wrong results), C5 share and C2,
# to price the fragmented byte stores.
set -o pipefail
mkdir -p gpurun_out
bash tools/ab_c5.sh base ${V2:-nopass} || exit 1
AB_CFGS="C2" bash tools/ab_cfgs.sh base ${V2:-nopass}
