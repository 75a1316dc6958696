#!/usr/bin/env bash
# Randomized soak: the seeded parity sweeps (tests/test_gpu_fuzz.py, tests/test_gpu_chain.py::test_chain_random)
# with many more seeds than the suite's default:  bash tools/gpu_soak.sh SEEDS [BASE]  (seeds BASE .. BASE + SEEDS - 1)
set -o pipefail
mkdir -p gpurun_out
SEEDS=${1:-200}
BASE=${2:-0}
RPT_FUZZ_SEED_BASE=$BASE RPT_FUZZ_SEEDS=$SEEDS timeout -k 10 1000 python -u -m pytest tests/test_gpu_fuzz.py "tests/test_gpu_chain.py::test_chain_random" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/soak.txt 2>&1 || { tail -40 gpurun_out/soak.txt; exit 1; }
tail -2 gpurun_out/soak.txt
