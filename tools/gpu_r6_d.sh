#!/usr/bin/env bash
# Full GPU tests + DBP15K bench and refinement timeline (top-k selection
# pairs) on HEAD.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6d; mkdir -p $O
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$O/$name.log" | cut -c1-300
  if [ $rc -ge 124 ]; then echo "FATAL $name $rc"; exit $rc; fi
  return 0
}
run topk 600 python -u -m pytest tests/test_hip_kernels.py -k topk -q -x --timeout 300 --timeout-method thread
run bench_topk 300 python -u tools/bench_topk_warm.py
run dbp 300 python bench.py --config dbp15k --steps 20 --warmup 3 --json-out $O/dbp.json
run prof 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --config dbp15k --kg-phase phase2 --steps 5 --warmup 2
f=$(find $O/prof -name '*kernel_trace.csv' | head -1); python tools/step_trace.py $f adam_multi 60 > $O/timeline_dbp_phase2.txt; rm -rf $O/prof
head -6 $O/timeline_dbp_phase2.txt | cut -c1-140
run pytest_gpu 1200 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
