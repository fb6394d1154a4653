#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6s; mkdir -p $O
timeout -k 10 600 python -u tools/bench_cu_reserve.py --hog 8 16 32 --reserve 8 16 32 --json $O/cu_reserve_r6.json > $O/cu.log 2>&1 || { tail -20 $O/cu.log; exit 1; }
cat $O/cu.log
