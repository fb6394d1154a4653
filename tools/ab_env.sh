#!/usr/bin/env bash
# Same-box A/B of bench.py, interleaved over two rounds.
#   tools/ab_env.sh STEPS "CFG_A" "CFG_B" ...
# CFG = environment assignments ("K=V K2=V2", may be empty); a leading
# "@base" runs the baseline worktree .ab_base/ (git worktree of an older
# commit with its own in-tree build) instead of this tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS=$1; shift
for round in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i + 1))
    script=bench.py
    envs=$cfg
    if [[ "$cfg" == @base* ]]; then
      script=.ab_base/bench.py
      envs=${cfg#@base}
    fi
    env $envs timeout -k 10 300 python "$script" --steps "$STEPS" --warmup 5 > gpurun_out/ab/run_${round}_$i.log 2>&1 || exit $?
    v=$(grep -o '"value": [0-9.]*' gpurun_out/ab/run_${round}_$i.log | head -1)
    echo "round $round [$cfg] $v"
  done
done
