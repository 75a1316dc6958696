#!/usr/bin/env bash
# Regenerate tests/golden/ from the Arrow Acero BlockedBloomFilter (pyarrow 25.0.0 wheel).
# TEST INFRASTRUCTURE ONLY: runs in the build container; needs pyarrow's headers and
# libarrow_acero.so.2500. Output is committed; nothing here runs on the GPU box.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
REPO="$(cd "$HERE/../.." && pwd)"
P="$(python3 -c 'import pyarrow, os; print(os.path.dirname(pyarrow.__file__))')"
OUT="${1:-$REPO/tests/golden}"
BUILD="$(mktemp -d)"
trap 'rm -rf "$BUILD"' EXIT
g++ -std=c++20 -O2 -I"$P/include" "$HERE/gen_arrow_golden.cc" -o "$BUILD/gen_arrow_golden" \
    -L"$P" -l:libarrow_acero.so.2500 -l:libarrow.so.2500 -Wl,-rpath,"$P"
mkdir -p "$OUT"
"$BUILD/gen_arrow_golden" "$OUT"
