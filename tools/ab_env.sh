#!/usr/bin/env bash
# Same-box A/B of bench.py under environment settings, interleaved.
#   tools/ab_env.sh STEPS "ENV_A" "ENV_B" [more...]   (each "K=V K2=V2" or "")
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS=$1; shift
for round in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i + 1))
    env $cfg timeout -k 10 300 python bench.py --steps "$STEPS" --warmup 5 > gpurun_out/ab/run_${round}_$i.log 2>&1 || exit $?
    v=$(grep -o '"value": [0-9.]*' gpurun_out/ab/run_${round}_$i.log | head -1)
    echo "round $round [$cfg] $v"
  done
done
