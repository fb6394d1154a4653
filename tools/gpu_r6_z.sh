#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6z; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_candidates.py tests/test_kg_trainer.py -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --config dbp15k --steps 20 --warmup 3 > $O/dbp.log 2>&1 || { tail -5 $O/dbp.log; exit 1; }
tail -1 $O/dbp.log | cut -c1-260
