set -o pipefail
V=$PWD/duckdb-robust-predicate-transfer_amd/build/variants
for v in skipz cur skipz cur; do echo "== $v"; RPT_GPU_LIB=$V/librpt_gpu_$v.so timeout -k 10 200 python tools/build_modes.py || exit 1; done
