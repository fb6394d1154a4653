#!/usr/bin/env bash
# Host AddressSanitizer + UBSan run of the native collator (csrc/host):
# builds tests/native/asan_collate.cpp + collate.cpp with
# -fsanitize=address,undefined against libtorch and runs it.  CPU only (GPU
# sanitizers are not available on this pool).
#   tools/asan_host.sh [build_dir]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-$ROOT/build/asan}
mkdir -p "$OUT"
read -r TINC TLIB ABI < <(python3 -c "
import os, torch
from torch.utils import cpp_extension as c
print(':'.join(c.include_paths()), os.path.join(os.path.dirname(torch.__file__), 'lib'), int(torch._C._GLIBCXX_USE_CXX11_ABI))")
INC=""
IFS=: read -ra PARTS <<< "$TINC"
for p in "${PARTS[@]}"; do INC="$INC -isystem $p"; done
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fopenmp \
  -fsanitize=address,undefined -fno-sanitize-recover=undefined \
  -D_GLIBCXX_USE_CXX11_ABI=$ABI $INC \
  "$ROOT/tests/native/asan_collate.cpp" "$ROOT/csrc/host/collate.cpp" \
  -L"$TLIB" -Wl,-rpath,"$TLIB" -ltorch_cpu -ltorch -lc10 \
  -o "$OUT/asan_collate"
# (detect_leaks=0: libtorch's static registries are reported as leaks)
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:verify_asan_link_order=0 \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 OMP_NUM_THREADS=4 \
  "$OUT/asan_collate"
