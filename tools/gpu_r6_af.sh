#!/usr/bin/env bash
# Stream-K top-k filter + the cheaper insertion rounds: tests, then a
# same-box A/B through two temporary host hooks (TK_AB_G fixes the
# workgroup count - 228 = the previous 76 row blocks x 3 equal target
# splits; TK_AB_OLD=1 launches the previous insertion rounds).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6af; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -k "topk or top_k or stream" -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "Error|assert|FAIL|rror" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
for cfg in "256 0" "228 1" "256 1" "228 0" "256 0" "228 1"; do
  set -- $cfg
  if [ "$2" = 1 ]; then export TK_AB_OLD=1; else unset TK_AB_OLD; fi
  TK_AB_G=$1 timeout -k 10 300 python -u tools/bench_topk_warm.py > $O/t_$1_$2.log 2>&1 || { tail -5 $O/t_$1_$2.log; exit 1; }
  echo "G=$1 old=$2 $(tail -1 $O/t_$1_$2.log | cut -c1-80)"
done
unset TK_AB_OLD
timeout -k 10 300 python bench.py --config dbp15k --steps 20 --warmup 3 > $O/dbp.log 2>&1 || { tail -5 $O/dbp.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*, "ms_per_step_phase1": [0-9.]*' $O/dbp.log
