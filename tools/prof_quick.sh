#!/usr/bin/env bash
# rocprofv3 kernel trace of a short bench run -> per-step kernel table.
#   tools/prof_quick.sh <name> [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
NAME=${1:-prof}; shift || true
OUT=$ROOT/gpurun_out/$NAME
rm -rf "$OUT"; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 "$ROOT/bench.py" --steps 6 --warmup 2 "$@" > "$OUT/log.txt" 2>&1 || exit $?
cd "$ROOT"
python3 tools/step_trace.py "$OUT/run_kernel_trace.csv" adam_multi 70 > "$OUT/step.txt"
python3 tools/step_trace.py "$OUT/run_kernel_trace.csv" adam_multi 0 --seq > "$OUT/seq.txt"
head -30 "$OUT/step.txt" | cut -c1-150
