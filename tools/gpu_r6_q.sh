#!/usr/bin/env bash
# DBP15K full-scale two-phase accuracy parity with the native psi_1 backward
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6q; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_relconv.py tests/test_gemm_tn.py -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 python -u tools/kg_parity.py --scale 1.0 --runs native,reference --out $O/kg_parity_full_r6.json > $O/kg.log 2>&1 || { tail -20 $O/kg.log; exit 1; }
tail -8 $O/kg.log
