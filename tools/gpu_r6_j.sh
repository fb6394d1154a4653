#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -k "topk" tests/test_relconv.py tests/test_kg_trainer.py tests/test_gemm_tn.py tests/test_gemm_f32.py -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "Error|assert|FAIL" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/bench_topk_warm.py > $O/bench_topk.log 2>&1 || { tail -5 $O/bench_topk.log; exit 1; }
cat $O/bench_topk.log
timeout -k 10 300 python bench.py --config dbp15k --steps 20 --warmup 3 --json-out $O/dbp.json > $O/dbp.log 2>&1 || { tail -5 $O/dbp.log; exit 1; }
tail -1 $O/dbp.log | cut -c1-330
for ph in phase1 phase2; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$ph -o run -- python bench.py --config dbp15k --kg-phase $ph --steps 5 --warmup 2 > $O/prof_$ph.log 2>&1 || { tail -5 $O/prof_$ph.log; exit 1; }
f=$(find $O/prof_$ph -name '*kernel_trace.csv' | head -1); python tools/step_trace.py $f adam_multi 60 > $O/timeline_dbp_$ph.txt || exit 1
rm -rf $O/prof_$ph
head -12 $O/timeline_dbp_$ph.txt | cut -c1-140
done
