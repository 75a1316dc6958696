# r03: count-free level 1, v1 (pool chunk per run boundary) vs v2 (fixed chunks + extents, deferred cursor use)
set -o pipefail
mkdir -p gpurun_out


bash tools/ab_c5.sh v1 v2 k0 k110
