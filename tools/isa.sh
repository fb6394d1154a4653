#!/usr/bin/env bash
# Device assembly of one HIP source (gfx950) for inspection:
#   tools/isa.sh csrc/hip/slot_gemm.hip > /tmp/slot_gemm.s
set -euo pipefail
cd "$(dirname "$0")/.."
CMD=$(grep -m1 "command = .*hipcc" build/native/build.ninja | sed 's/^ *command = //; s/-MD -MF \$out.d -c \$in -o \$out//')
$CMD --offload-device-only -S -o - "$1"
