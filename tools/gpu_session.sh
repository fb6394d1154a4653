#!/usr/bin/env bash
# One GPU-box session: tests -> smoke -> bench (native / reference) -> optional
# rocprofv3 kernel stats.  Each GPU step has its own time limit; the script
# stops at the first crash/timeout (exit >= 124) but continues after ordinary
# test failures so one call yields as much evidence as possible.
#
#   tools/gpu_session.sh [tests] [smoke] [bench] [ref] [prof] [scale]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS="${STEPS:-20}"
WARM="${WARM:-5}"

run() {  # run <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "$OUT/$name.log"
  if [ $rc -ge 124 ]; then
    echo "FATAL: $name exited with $rc; stopping GPU work in this call"
    exit $rc
  fi
  return 0
}

want() { [ $# -eq 0 ] && return 0; for a in "${ARGS[@]}"; do [ "$a" = "$1" ] && return 0; done; return 1; }
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(tests smoke bench ref)

want tests && run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
want smoke && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
want bench && run bench_native 600 python bench.py --steps "$STEPS" --warmup "$WARM" --json-out "$OUT/bench_native.json"
want ref && run bench_reference 900 python bench.py --impl reference --steps "$((STEPS / 2 > 3 ? STEPS / 2 : 3))" --warmup 2 --json-out "$OUT/bench_reference.json"
if want prof; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  run rocprof 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --steps 5 --warmup 2
fi
want torchprof && run torchprof 600 python tools/profile_step.py --steps 2 --rows 60
echo "=== done ($(date +%T))"
