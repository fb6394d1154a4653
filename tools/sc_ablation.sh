#!/usr/bin/env bash
# Ablation / timing sweep of the fused slot conv (tools/bench_slot_conv.py).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for d in ${SC_DEBUG_SET:-0 1 2 4 7}; do
  DGMC_SC_DEBUG=$d timeout -k 10 120 python tools/bench_slot_conv.py >> gpurun_out/sc_abl.log 2>&1
done
