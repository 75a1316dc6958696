set -o pipefail
mkdir -p gpurun_out
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
for v in bsl9 bsl10; do
RPT_GPU_LIB=$V/librpt_gpu_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_bucketed.py -k "c5_geometry" > gpurun_out/t_$v.txt 2>&1 || { tail -20 gpurun_out/t_$v.txt; exit 1; }
tail -1 gpurun_out/t_$v.txt
done
AB_CFGS="C5" bash tools/ab_cfgs.sh bsl8 bsl9 bsl10
