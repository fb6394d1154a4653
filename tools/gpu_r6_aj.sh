#!/usr/bin/env bash
# Top-k merge-tile count re-checked after the cheaper insertion rounds
# (TK_AB_MT: a temporary host hook selecting the kernel instantiation, since
# removed: kX3MergeTiles = 2).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6aj; mkdir -p $O
for mt in 2 1 2 1 2 1; do
  TK_AB_MT=$mt timeout -k 10 300 python -u tools/bench_topk_warm.py > $O/t_$mt.log 2>&1 || { tail -5 $O/t_$mt.log; exit 1; }
  echo "mt=$mt $(tail -1 $O/t_$mt.log | cut -c1-60)"
done
