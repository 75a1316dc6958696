# r03: level-2 metadata loads issued before the early-exit test (partition chunk map + tile count, unpermute)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bucketed.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ab7.txt 2>&1 || { tail -40 gpurun_out/t_ab7.txt; exit 1; }
tail -1 gpurun_out/t_ab7.txt
bash tools/ab_c5.sh head base && bash tools/ab_c5.sh head base
