# r03: unpermute kernels: pass bits as 32-bit words from a static LDS array, pairwise bfe extraction
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ab8.txt 2>&1 || { tail -40 gpurun_out/t_ab8.txt; exit 1; }
tail -1 gpurun_out/t_ab8.txt
AB_CFGS="C2 C3" bash tools/ab_cfgs.sh head base && bash tools/ab_c5.sh head base
