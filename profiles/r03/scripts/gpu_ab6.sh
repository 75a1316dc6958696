# r03: min/max published once per workgroup (bucket scatter, partition): build time, HEAD vs working tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_minmax_composite.py tests/test_gpu_bucketed.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ab6.txt 2>&1 || { tail -40 gpurun_out/t_ab6.txt; exit 1; }
tail -1 gpurun_out/t_ab6.txt
bash tools/ab_c5.sh head base && AB_CFGS="C3 C2" bash tools/ab_cfgs.sh head base
