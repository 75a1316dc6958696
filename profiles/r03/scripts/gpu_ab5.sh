# r03: min/max publish once per scatter workgroup (build); bucket unpermute workgroup size (probe)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bucketed.py tests/test_gpu_minmax_composite.py tests/test_gpu_deferred_clear.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ab5.txt 2>&1 || { tail -40 gpurun_out/t_ab5.txt; exit 1; }
tail -1 gpurun_out/t_ab5.txt
bash tools/ab_c5.sh base u512 u1024
