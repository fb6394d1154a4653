#!/usr/bin/env bash
# Round evidence on one GPU box: full GPU test suite, smoke, 200-step fp32
# bench (headline), bf16 bench (extra), rocprofv3 kernel stats + one-step
# timeline of the fp32 step.  Each GPU step has its own time limit; the
# script stops at the first failure.
#   tools/gpu_evidence.sh <tag>
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-ev}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 \
  --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1
timeout -k 10 300 python bench.py --steps 200 --warmup 20 \
  --json-out "$OUT/bench_fp32.json" > "$OUT/bench_fp32.log" 2>&1
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --dtype bf16 \
  --json-out "$OUT/bench_bf16.json" > "$OUT/bench_bf16.log" 2>&1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$OUT/prof" -o run -- python bench.py --steps 5 --warmup 2 \
  --eval-pairs 0 > "$OUT/prof.log" 2>&1
python3 tools/kstats.py "$OUT/prof/run_kernel_stats.csv" 15 60 \
  > "$OUT/kstats.txt"
python3 tools/step_trace.py "$OUT/prof/run_kernel_trace.csv" \
  adam_multi_kernel > "$OUT/step.txt"
echo "evidence done $TAG"
