#!/usr/bin/env bash
# Joint planes from the transport kernels: tests, then a same-box A/B of the
# PascalVOC step (B: psi_2 input split by split3 as before, via a
# monkeypatch of SplineCNN.takes_x6_planes), then a step timeline.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6ad; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -k "step or planes or fused" -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u -m pytest tests/test_slot_gemm.py tests/test_slot_gemm_x6.py -q -x --timeout 300 --timeout-method thread > $O/pytest2.log 2>&1 || { grep -E "Error|assert|FAIL" $O/pytest2.log | head -20; exit 1; }
tail -1 $O/pytest2.log
B="import sys; sys.argv=['bench.py','--steps','100','--warmup','10']; from deep_graph_matching_consensus_amd.models import SplineCNN; SplineCNN.takes_x6_planes=lambda s, x: False; import runpy; runpy.run_path('bench.py', run_name='__main__')"
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 > $O/a_$i.log 2>&1 || { tail -5 $O/a_$i.log; exit 1; }
  echo "A(planes) $(grep -o '"ms_per_step": [0-9.]*' $O/a_$i.log)"
  timeout -k 10 300 python -c "$B" > $O/b_$i.log 2>&1 || { tail -5 $O/b_$i.log; exit 1; }
  echo "B(split)  $(grep -o '"ms_per_step": [0-9.]*' $O/b_$i.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1); python tools/step_trace.py $f adam_multi 80 > $O/timeline.txt; rm -rf $O/prof
head -3 $O/timeline.txt | cut -c1-140; grep -c split3 $O/timeline.txt || true
