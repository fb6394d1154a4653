#!/usr/bin/env bash
# rocprofv3 kernel trace of a short bench run + per-step timeline summary.
#   tools/prof_step.sh [name] [extra bench args...]
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
NAME=${1:-prof}; shift || true
OUT=$ROOT/gpurun_out/$NAME
rm -rf "$OUT"; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 "$ROOT/bench.py" --steps 6 --warmup 2 "$@" > "$OUT/log.txt" 2>&1
cd "$ROOT"
grep '"metric"' "$OUT/log.txt" || true
python3 tools/step_trace.py "$OUT/run_kernel_trace.csv" adam_multi_kernel 60 > "$OUT/step.txt"
python3 tools/step_trace.py "$OUT/run_kernel_trace.csv" adam_multi_kernel 0 --seq > "$OUT/seq.txt"
head -45 "$OUT/step.txt"
