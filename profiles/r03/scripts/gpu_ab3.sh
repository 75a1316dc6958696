# r03 A/B: count-free bucketed level 1 -- tile size, scatter copy-out cost, list groups (C5 share)
set -o pipefail
bash tools/ab_c5.sh base t8k sk1 sk3 || exit 1
bash tools/ab_env.sh "--build-rows 1e9 --filter-rows 8e9" "-" "RPT_L1_GROUPS_MIN_ROWS=100000000000"
