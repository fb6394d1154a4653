#!/usr/bin/env bash
# (Round-6 A/B of the top-k first-tile sort: TK_AB_NOSORT was a temporary
# host hook of that build, removed after the measurement.)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6ab; mkdir -p $O
for v in sort nosort sort nosort; do
  if [ $v = nosort ]; then export TK_AB_NOSORT=1; else unset TK_AB_NOSORT; fi
  timeout -k 10 300 python -u tools/bench_topk_warm.py > $O/t_$v.log 2>&1 || { tail -5 $O/t_$v.log; exit 1; }
  echo "$v $(tail -1 $O/t_$v.log | cut -c1-60)"
done
unset TK_AB_NOSORT
timeout -k 10 300 python bench.py --config dbp15k --steps 20 --warmup 3 > $O/dbp_sort.log 2>&1 && echo "sort $(tail -1 $O/dbp_sort.log | cut -c60-200)"
TK_AB_NOSORT=1 timeout -k 10 300 python bench.py --config dbp15k --steps 20 --warmup 3 > $O/dbp_nosort.log 2>&1 && echo "nosort $(tail -1 $O/dbp_nosort.log | cut -c60-200)"
