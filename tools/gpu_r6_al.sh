#!/usr/bin/env bash
# Top-k filter at C = 256 with 4-wave workgroups (two per CU, barriers over
# 4 waves, each target tile serving 128 rows) vs 8-wave ones (TK_AB_W4: a
# temporary host hook, since removed; its first version also forced W = 4
# onto the C <= 128 kernels, a launch / kernel mismatch that faulted - fixed
# before the measured run).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6al; mkdir -p $O
TK_AB_W4=1 timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -k "topk or top_k or split_shapes" -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "Error|assert|FAIL|rror" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
for w in 8 4 8 4 8 4; do
  if [ "$w" = 4 ]; then export TK_AB_W4=1; else unset TK_AB_W4; fi
  timeout -k 10 300 python -u tools/bench_topk_warm.py > $O/t_$w.log 2>&1 || { tail -5 $O/t_$w.log; exit 1; }
  echo "W=$w $(tail -1 $O/t_$w.log | cut -c1-60)"
done
