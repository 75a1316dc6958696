set -o pipefail
bash tools/gpu_check.sh selx || exit 1
bash tools/ab_args.sh "--config C2 --p 0.1|--config C2 --p 0.25|--config C2 --p 0.5|--config C2 --p 1.0|--config C5 --p 0.1|--config C5 --p 0.5" oldsel m64 m128 m192
