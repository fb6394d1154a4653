#!/usr/bin/env bash
# Full GPU check of HEAD: pytest -m gpu, smoke, PascalVOC + DBP15K benches,
# one-step PascalVOC kernel timeline.  Stops at the first crash/timeout.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6full; mkdir -p $O
run() {  # run <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$O/$name.log" | cut -c1-300
  if [ $rc -ge 124 ]; then echo "FATAL $name $rc"; exit $rc; fi
  return 0
}
run pytest_gpu 1000 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run pascal 300 python bench.py --steps 100 --warmup 10 --json-out $O/pascal.json
run dbp 300 python bench.py --config dbp15k --steps 20 --warmup 3 --json-out $O/dbp.json
run prof 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5
f=$(find $O/prof -name '*kernel_trace.csv' | head -1); python tools/step_trace.py $f adam_multi 60 > $O/timeline_pascal.txt; rm -rf $O/prof
head -30 $O/timeline_pascal.txt | cut -c1-140
