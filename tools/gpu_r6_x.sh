#!/usr/bin/env bash
# Reproduce the round-6 final-run failure: the GPU tests in suite order up
# to test_gemm_tn.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6x; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_candidates.py tests/test_checkpoint.py tests/test_datasets.py tests/test_determinism.py tests/test_device_loader.py tests/test_dgmc.py tests/test_distributed.py tests/test_dp_step.py tests/test_encoders.py tests/test_failures.py tests/test_gemm_f32.py tests/test_gemm_tn.py -m gpu -q -rf --timeout 300 --timeout-method thread > $O/p.log 2>&1; echo "rc=$?"
grep -E "passed|failed|AssertionError|^E  " $O/p.log | head -20 | cut -c1-600
