#!/usr/bin/env bash
# Quick GPU check: selected tests (pytest -k expression $1) + a bench run.
#   tools/quick_session.sh "<pytest -k expr>" [bench steps]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/q
export HSA_ENABLE_IPC_MODE_LEGACY=0
K="${1:-}"
STEPS="${2:-100}"
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/q/tests.log 2>&1
  rc=$?; tail -4 gpurun_out/q/tests.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ "$STEPS" != "0" ]; then
  timeout -k 10 300 python bench.py --steps "$STEPS" --warmup 5 > gpurun_out/q/bench.log 2>&1
  rc=$?; tail -1 gpurun_out/q/bench.log | cut -c1-220
  exit $rc
fi
