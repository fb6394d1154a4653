#!/usr/bin/env bash
# A/B: psi_1 layer-0 dY_c as planes (no dX reader) vs fp32
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6v; mkdir -p $O
run() {  # $1 = True/False
timeout -k 10 300 python -c "
import sys, runpy
import deep_graph_matching_consensus_amd.ops.slot_gemm as sg
sg.DY_PLANES_NO_DX = $1
sys.argv = ['bench.py', '--steps', '100', '--warmup', '10']
runpy.run_path('bench.py', run_name='__main__')" > $O/bench_$1.log 2>&1 || { tail -5 $O/bench_$1.log; exit 1; }
echo "$1 $(tail -1 $O/bench_$1.log | cut -c1-150)"
}
timeout -k 10 600 python -u -m pytest tests/test_slot_gemm_x6.py tests/test_slot_gemm.py -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
run True && run False && run True && run False
