#!/usr/bin/env bash
# Round-6 HEAD record on one box: pytest -m gpu, smoke, every config's bench,
# PascalVOC and DBP15K (both phases, refinement step last) timelines.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${R6FINAL_DIR:-r6final}; mkdir -p $O
run() {  # run <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 2 "$O/$name.log" | cut -c1-260
  if [ $rc -ge 124 ]; then echo "FATAL $name $rc"; exit $rc; fi
  return 0
}
run pytest_gpu 1100 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run pascal_driver 300 python bench.py --json-out $O/pascal_driver.json
run pascal 300 python bench.py --steps 100 --warmup 10 --json-out $O/pascal.json
run willow 300 python bench.py --config willow --steps 100 --warmup 10 --json-out $O/willow.json
run dbp15k 300 python bench.py --config dbp15k --steps 20 --warmup 3 --json-out $O/dbp15k.json
run sinkhorn 300 python bench.py --normalization sinkhorn --steps 100 --warmup 10 --json-out $O/sinkhorn.json
run bf16 300 python bench.py --dtype bf16 --steps 100 --warmup 10 --json-out $O/bf16.json
run prof 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5
f=$(find $O/prof -name '*kernel_trace.csv' | head -1); python tools/step_trace.py $f adam_multi 80 > $O/timeline_pascal.txt; rm -rf $O/prof
run profk 300 rocprofv3 --kernel-trace --output-format csv -d $O/profk -o run -- python bench.py --config dbp15k --steps 5 --warmup 2
f=$(find $O/profk -name '*kernel_trace.csv' | head -1); python tools/step_trace.py $f adam_multi 80 > $O/timeline_dbp15k.txt; rm -rf $O/profk
head -3 $O/timeline_pascal.txt | cut -c1-140; head -3 $O/timeline_dbp15k.txt | cut -c1-140
