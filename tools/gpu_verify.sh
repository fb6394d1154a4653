#!/usr/bin/env bash
# Session check: GPU tests on HEAD, then the native-vs-reference accuracy
# parity run (200 steps).  Each step has its own limit; stop at the first
# failure.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/verify
mkdir -p "$OUT"
want() { for a in "${ARGS[@]}"; do [ "$a" = "$1" ] && return 0; done; return 1; }
ARGS=("$@")
if want tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 \
    --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  tail -3 "$OUT/pytest_gpu.log"
fi
if want smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" \
    > "$OUT/smoke.log" 2>&1
fi
if want parity; then
  timeout -k 10 900 python -u tools/parity_run.py --steps 200 \
    --out "$OUT/accuracy_parity.json" > "$OUT/parity.log" 2>&1
fi
if want bench; then
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 \
    --json-out "$OUT/bench_fp32.json" > "$OUT/bench_fp32.log" 2>&1
  tail -1 "$OUT/bench_fp32.log"
fi
echo "verify done"
