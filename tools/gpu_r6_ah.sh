#!/usr/bin/env bash
# Top-k A/B through a temporary host hook (TK_AB_OLD=1: the previous
# kernel); first use: sorted-prefix insertion test, second: tile pre-check
# only in warm mode, third: column mask applied to the votes once a tile,
# fourth: DPP shifts without an "old" operand + ballot masked in scalar,
# fifth: bitonic partner exchanges by DPP for lane distances 1, 2, 8.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6ah; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -k "topk or top_k or split_shapes" -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "Error|assert|FAIL|rror" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
for old in 0 1 0 1 0 1; do
  if [ "$old" = 1 ]; then export TK_AB_OLD=1; else unset TK_AB_OLD; fi
  timeout -k 10 300 python -u tools/bench_topk_warm.py > $O/t_$old.log 2>&1 || { tail -5 $O/t_$old.log; exit 1; }
  echo "old=$old $(tail -1 $O/t_$old.log | cut -c1-60)"
done
