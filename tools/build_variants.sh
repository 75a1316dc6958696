#!/usr/bin/env bash
# Build librpt_gpu.so variants with different compile-time tuning macros for A/B timing on the box:
#   bash tools/build_variants.sh "u4:-DRPT_SLICE_UNROLL=4" "s13:-DRPT_SLICE_LOG=13" ...
# Output: duckdb-robust-predicate-transfer_amd/build/variants/librpt_gpu_<name>.so (select with RPT_GPU_LIB).
set -eu
PKG=duckdb-robust-predicate-transfer_amd
OUT=$PKG/build/variants
mkdir -p "$OUT"
make -C $PKG build/rpt_host.o >/dev/null
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  (
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $flags \
      -Iinclude -I$PKG/csrc -c $PKG/csrc/rpt_gpu.hip -o "$OUT/rpt_gpu_$name.o" &&
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/librpt_gpu_$name.so" "$OUT/rpt_gpu_$name.o" $PKG/build/rpt_host.o &&
    echo "built $name ($flags)"
  ) &
done
wait
