#!/usr/bin/env bash
# Kernel-trace profiles of this tree and of the .ab_base worktree (same box)
# -> gpurun_out/<name>_{cur,base}/step.txt for a per-kernel diff.
#   tools/prof_ab.sh <name>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
NAME=${1:-pab}
export HSA_ENABLE_IPC_MODE_LEGACY=0
for which in cur base; do
  OUT=$ROOT/gpurun_out/${NAME}_$which
  rm -rf "$OUT"; mkdir -p "$OUT"
  BENCH=$ROOT/bench.py
  [ "$which" = base ] && BENCH=$ROOT/.ab_base/bench.py
  (cd /tmp && TMPDIR=/tmp timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 "$BENCH" --steps 6 --warmup 2 > "$OUT/log.txt" 2>&1) || exit $?
  python3 tools/step_trace.py "$OUT/run_kernel_trace.csv" adam_multi 70 > "$OUT/step.txt"
  python3 tools/step_trace.py "$OUT/run_kernel_trace.csv" adam_multi 0 --seq > "$OUT/seq.txt"
  head -1 "$OUT/step.txt"
done
