#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6i; mkdir -p $O
for i in 1 2 3; do
timeout -k 10 600 python -u -m pytest tests/test_gemm_tn.py -q -x --timeout 300 --timeout-method thread > $O/pytest$i.log 2>&1 || { grep -E "Error|assert" $O/pytest$i.log | head; exit 1; }
tail -1 $O/pytest$i.log
done
timeout -k 10 300 python -u tools/bench_gemm_tn.py --cfgs 0 3 4 5 --no-torch --json $O/bench_tn.json > $O/bench_tn.log 2>&1 || { tail -20 $O/bench_tn.log; exit 1; }
cat $O/bench_tn.log
