#!/usr/bin/env bash
# Per-core speed of the CPU restatement (the bench's cpu_baseline "port") against Arrow Acero's
# BlockedBloomFilter::Find on the same filter and hashes. TEST INFRASTRUCTURE ONLY: runs in
# the build container (pyarrow 25.0.0), never on the GPU box.
#   bash oracle/arrow_golden/cpu_crosscheck.sh [OUT]      (default: print to stdout)
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
REPO="$(cd "$HERE/../.." && pwd)"
P="$(python3 -c 'import pyarrow, os; print(os.path.dirname(pyarrow.__file__))')"
make -C "$REPO/oracle" >/dev/null
BUILD="$(mktemp -d)"
trap 'rm -rf "$BUILD"' EXIT
g++ -std=c++20 -O2 -I"$P/include" "$HERE/cpu_crosscheck.cc" -o "$BUILD/cpu_crosscheck" \
    -L"$P" -l:libarrow_acero.so.2500 -l:libarrow.so.2500 -L"$REPO/oracle/build" -lrpt_oracle \
    -Wl,-rpath,"$P" -Wl,-rpath,"$REPO/oracle/build"
{
  echo "# $(lscpu | sed -n 's/^Model name: *//p')"
  "$BUILD/cpu_crosscheck"
} | tee ${1:-/dev/null}
