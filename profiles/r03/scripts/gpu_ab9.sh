#!/usr/bin/env bash
# r03: the bucketed probe's fused sel tail (level-1 tile counts -> offsets -> bucket_unpermute writes the sel)
# vs the result-bit tail + compaction: GPU tests, then C5-share and C2 A/B of the HEAD build ("base") and the
# working tree ("fused").
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bucketed.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ab9.txt 2>&1 || { tail -40 gpurun_out/t_ab9.txt; exit 1; }
tail -2 gpurun_out/t_ab9.txt
bash tools/ab_c5.sh base fused || exit 1
AB_CFGS="C2" bash tools/ab_cfgs.sh base fused
