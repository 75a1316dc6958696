#!/usr/bin/env bash
# Build librpt_gpu.so from the sources of a git revision, as an A/B variant next to the working tree's:
#   bash tools/build_rev_variant.sh NAME REV     -> duckdb-robust-predicate-transfer_amd/build/variants/librpt_gpu_NAME.so
set -eu
NAME=$1; REV=$2
PKG=duckdb-robust-predicate-transfer_amd
SRC=$PKG/build/rev_$NAME
OUT=$PKG/build/variants
rm -rf "$SRC"; mkdir -p "$SRC/kernels" "$SRC/include" "$OUT"
for f in $(git ls-tree -r --name-only "$REV" $PKG/csrc include); do
  case $f in
    $PKG/csrc/*) git show "$REV:$f" > "$SRC/${f#$PKG/csrc/}" ;;
    include/*) git show "$REV:$f" > "$SRC/include/${f#include/}" ;;
  esac
done
make -C $PKG build/rpt_host.o >/dev/null
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I"$SRC/include" -I"$SRC" \
  -c "$SRC/rpt_gpu.hip" -o "$SRC/rpt_gpu.o"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/librpt_gpu_$NAME.so" "$SRC/rpt_gpu.o" $PKG/build/rpt_host.o
rm -rf "$SRC"
echo "built $OUT/librpt_gpu_$NAME.so from $REV"
