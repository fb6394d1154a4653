#!/usr/bin/env bash
# ReLU/bias backward hand-off: tests + PascalVOC bench + timeline
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_slot_gemm.py tests/test_slot_gemm_x6.py tests/test_dgmc.py tests/test_loopgrad.py tests/test_grad_pieces.py tests/test_determinism.py -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --json-out $O/pascal.json > $O/pascal.log 2>&1 || { tail -5 $O/pascal.log; exit 1; }
tail -1 $O/pascal.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --steps 5 --warmup 2 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1); python tools/step_trace.py $f adam_multi 80 > $O/timeline.txt && python tools/step_trace.py $f adam_multi 400 --seq > $O/seq.txt || exit 1
rm -rf $O/prof
head -3 $O/timeline.txt | cut -c1-150
grep -E "colsum|gather_sum" $O/timeline.txt | cut -c1-120
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/profk -o run -- python bench.py --config dbp15k --kg-phase phase2 --steps 5 --warmup 2 > $O/profk.log 2>&1 || { tail -5 $O/profk.log; exit 1; }
f=$(find $O/profk -name '*kernel_trace.csv' | head -1); python tools/step_trace.py $f adam_multi 60 > $O/timeline_dbp.txt && python tools/step_trace.py $f adam_multi 400 --seq > $O/seq_dbp.txt || exit 1
rm -rf $O/profk
head -8 $O/timeline_dbp.txt | cut -c1-140
grep -E "spmm_piece_fold" $O/timeline_dbp.txt | cut -c1-120
