#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_tn.py tests/test_gemm_f32.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -u tools/bench_gemm_tn.py --cfgs 0 4 5 --no-torch --json $O/bench_tn.json > $O/bench_tn.log 2>&1 || { tail -20 $O/bench_tn.log; exit 1; }
cat $O/bench_tn.log
timeout -k 10 300 python -u tools/bench_gemm_nt.py --json $O/bench_nt.json > $O/bench_nt.log 2>&1 || { tail -20 $O/bench_nt.log; exit 1; }
cat $O/bench_nt.log
