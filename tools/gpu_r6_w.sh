#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_f32.py tests/test_gemm_tn.py -q -rf --timeout 300 --timeout-method thread > $O/p1.log 2>&1; echo "rc=$?"; tail -3 $O/p1.log
timeout -k 10 600 python -u -m pytest tests/test_gemm_tn.py -q -rf --timeout 300 --timeout-method thread > $O/p2.log 2>&1; echo "rc=$?"; tail -3 $O/p2.log
