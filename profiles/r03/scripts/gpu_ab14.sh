#!/usr/bin/env bash
# r03: pass bytes written slice-major by the slice probe, then a blocked transpose to tile-major (instead of
# partial-line byte stores into the tile-major array): GPU parity tests, then C5-share / C2 / C3 A/B against
# HEAD's build.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bucketed.py tests/test_gpu_fuzz.py tests/test_gpu_chain.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ab14.txt 2>&1 || { tail -40 gpurun_out/t_ab14.txt; exit 1; }
tail -1 gpurun_out/t_ab14.txt
bash tools/ab_c5.sh base sm || exit 1
AB_CFGS="C2 C3" bash tools/ab_cfgs.sh base sm
