#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_tn.py tests/test_gemm_f32.py -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "AssertionError|assert |passed|failed" $O/pytest.log | head -30
