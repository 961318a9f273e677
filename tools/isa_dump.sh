#!/bin/bash
# Device assembly of every library source, as the Makefile builds it (same flags), into $1
# (default /tmp/isa): used to check that a source clean-up leaves the default code objects
# unchanged (diff -r of two dumps; comment and .ident lines dropped).
#   tools/isa_dump.sh /tmp/isa_before   ...edit...   tools/isa_dump.sh /tmp/isa_after
set -euo pipefail
OUT=${1:-/tmp/isa}
CSRC=$(cd "$(dirname "$0")/../tensor_regression_amd/csrc" && pwd)
mkdir -p "$OUT"
cd "$CSRC"
make -s build/tr_build_id.h
for f in *.hip; do
  extra=""
  case $f in
    tr_mnl_duo.hip) extra="-fno-slp-vectorize -fno-honor-nans" ;;
    tr_spectral_slice.hip) extra="-fno-slp-vectorize" ;;
  esac
  # shellcheck disable=SC2086
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function $extra -Ibuild \
    --cuda-device-only -S "$f" -o - 2>/dev/null |
    grep -v -E '^\s*(;|//|\.ident|\.file|\.loc)' > "$OUT/${f%.hip}.s" &
done
wait
wc -l "$OUT"/*.s | tail -1
