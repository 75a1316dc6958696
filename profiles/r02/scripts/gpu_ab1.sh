set -o pipefail
mkdir -p gpurun_out
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_minmax_composite.py tests/test_gpu_bucketed.py > gpurun_out/t_dpp.txt 2>&1 || { tail -20 gpurun_out/t_dpp.txt; exit 1; }
tail -2 gpurun_out/t_dpp.txt
RPT_GPU_LIB=$V/librpt_gpu_bsl8.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_bucketed.py -k "c5_geometry" > gpurun_out/t_bsl8.txt 2>&1 || { tail -20 gpurun_out/t_bsl8.txt; exit 1; }
tail -2 gpurun_out/t_bsl8.txt
AB_CFGS="C5" bash tools/ab_cfgs.sh base dpp bsl8 && AB_CFGS="C3" bash tools/ab_cfgs.sh base dpp
