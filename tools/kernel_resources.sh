#!/usr/bin/env bash
# Per-kernel VGPR / LDS / occupancy of one HIP source (compile-time remarks).
#   tools/kernel_resources.sh csrc/hip/dense_consensus.hip [name-filter]
set -e
SRC=$1; FILTER=${2:-.}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
INC=$(python3 -c "from torch.utils import cpp_extension as c; print(' '.join('-isystem '+p for p in c.include_paths(device_type='cuda')))")
ABI=$(python3 -c "import torch; print(int(torch._C._GLIBCXX_USE_CXX11_ABI))")
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -D_GLIBCXX_USE_CXX11_ABI=$ABI \
  -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 $INC -x hip --offload-arch=gfx950 \
  -fno-gpu-rdc --cuda-device-only -I"$ROOT/csrc/hip" -c "$ROOT/$SRC" \
  -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size" |
  sed -e 's/.*remark: //' | paste - - - - - - | grep -E "$FILTER" |
  sed -e 's/\[-Rpass-analysis=kernel-resource-usage\]//g' | cut -c1-220
