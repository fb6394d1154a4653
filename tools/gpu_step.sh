#!/usr/bin/env bash
# One focused GPU-box session for the PascalVOC flagship:
#   tools/gpu_step.sh <tag> [pytest-args...]
# runs the given GPU tests (if any), the default bench (fp32) and a
# rocprofv3 kernel-stats profile into gpurun_out/<tag>_*.  Every GPU step has
# its own time limit; the script stops at the first failure.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-run}; shift || true
OUT=gpurun_out
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -v --timeout 120 \
    --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1
fi
timeout -k 10 300 python bench.py --steps "${STEPS:-20}" --warmup "${WARM:-5}" \
  ${BENCH_ARGS:-} --json-out "$OUT/${TAG}_bench.json" > "$OUT/${TAG}_bench.log" 2>&1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$OUT/${TAG}_prof" -o run -- python bench.py --steps 5 --warmup 2 \
  --eval-pairs 0 ${BENCH_ARGS:-} > "$OUT/${TAG}_prof.log" 2>&1
echo "done $TAG"
