#!/usr/bin/env bash
# psi_1 layer-0 weight-gradient rounds (ops/slot_gemm.py X6_WGRAD_ROUNDS_BIG,
# set by a monkeypatch before bench.py runs): PascalVOC 100-step, same box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6ai; mkdir -p $O
for r in 6 3 4 8 6 3 4 8; do
  timeout -k 10 300 python -c "import sys; sys.argv=['bench.py','--steps','100','--warmup','10']; from deep_graph_matching_consensus_amd.ops import slot_gemm; slot_gemm.X6_WGRAD_ROUNDS_BIG=$r; import runpy; runpy.run_path('bench.py', run_name='__main__')" > $O/r_$r.log 2>&1 || { tail -5 $O/r_$r.log; exit 1; }
  echo "rounds=$r $(grep -o '"ms_per_step": [0-9.]*' $O/r_$r.log)"
done
