#!/usr/bin/env bash
# top-k lane lists: tests, filter timing, DBP15K bench; then KG accuracy parity
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -k "topk" -q -x --timeout 300 --timeout-method thread > $O/pytest_topk.log 2>&1 || { grep -E "Error|assert|FAIL" $O/pytest_topk.log | head -20; exit 1; }
tail -1 $O/pytest_topk.log
timeout -k 10 300 python -u tools/bench_topk_warm.py > $O/bench_topk.log 2>&1 || { tail -5 $O/bench_topk.log; exit 1; }
cat $O/bench_topk.log
timeout -k 10 300 python bench.py --config dbp15k --steps 20 --warmup 3 --json-out $O/dbp.json > $O/dbp.log 2>&1 || { tail -5 $O/dbp.log; exit 1; }
tail -1 $O/dbp.log | cut -c1-330
timeout -k 10 600 python -u -m pytest tests/test_relconv.py tests/test_gemm_tn.py tests/test_kg_trainer.py tests/test_candidates.py -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 python -u tools/kg_parity.py --scale 1.0 --runs native,reference --out $O/kg_parity_full_r6.json > $O/kg.log 2>&1 || { tail -20 $O/kg.log; exit 1; }
tail -8 $O/kg.log
