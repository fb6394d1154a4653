#!/usr/bin/env bash
# (A/B of the top-k merge-tile count through a temporary host hook, TK_AB_MERGE,
#  since removed: the kernel now fixes kX3MergeTiles = 4; rerunning this
#  script times the same kernel for every m)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6ac; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -k "topk" -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
for m in 1 2 4 6 8 1 4; do
  TK_AB_MERGE=$m timeout -k 10 300 python -u tools/bench_topk_warm.py > $O/t_$m.log 2>&1 || { tail -5 $O/t_$m.log; exit 1; }
  echo "merge=$m $(tail -1 $O/t_$m.log | cut -c1-40)"
done
