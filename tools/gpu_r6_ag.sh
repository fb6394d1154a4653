#!/usr/bin/env bash
# Top-k filter with the cheaper insertion rounds (equal target splits):
# tests, the filter bench, the DBP15K bench and its step timeline.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6ag; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -k "topk or top_k or split_shapes" -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "Error|assert|FAIL|rror" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/bench_topk_warm.py --json $O/topk.json > $O/t.log 2>&1 || { tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log | cut -c1-200
timeout -k 10 300 python bench.py --config dbp15k --steps 20 --warmup 3 --json-out $O/dbp15k.json > $O/dbp.log 2>&1 || { tail -5 $O/dbp.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*, "ms_per_step_phase1": [0-9.]*' $O/dbp.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/profk -o run -- python bench.py --config dbp15k --steps 5 --warmup 2 > $O/profk.log 2>&1 || { tail -5 $O/profk.log; exit 1; }
f=$(find $O/profk -name '*kernel_trace.csv' | head -1); python tools/step_trace.py $f adam_multi 80 > $O/timeline_dbp15k.txt; rm -rf $O/profk
head -4 $O/timeline_dbp15k.txt | cut -c1-140
