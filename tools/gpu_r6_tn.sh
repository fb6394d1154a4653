#!/usr/bin/env bash
# Round 6: native psi_1 backward (TN / masked NT GEMMs) + warm-started top-k
# filter - numerics tests, micro-benchmark, DBP15K bench and timelines.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6tn; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gemm_tn.py tests/test_gemm_f32.py tests/test_relconv.py tests/test_kg_trainer.py "tests/test_hip_kernels.py::test_topk_warm_start_same_output" "tests/test_hip_kernels.py::test_topk_exact_refined_equals_brute_force" "tests/test_hip_kernels.py::test_topk_nonfinite_rows_give_valid_indices" -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -u tools/bench_gemm_tn.py --json $O/bench_tn.json > $O/bench_tn.log 2>&1 || { tail -20 $O/bench_tn.log; exit 1; }
cat $O/bench_tn.log
timeout -k 10 300 python bench.py --config dbp15k --steps 20 --warmup 3 > $O/dbp.log 2>&1 || { tail -20 $O/dbp.log; exit 1; }
tail -1 $O/dbp.log | cut -c1-400
for ph in phase1 phase2; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$ph -o run -- python bench.py --config dbp15k --kg-phase $ph --steps 5 --warmup 2 > $O/prof_$ph.log 2>&1 || { tail -20 $O/prof_$ph.log; exit 1; }
f=$(find $O/prof_$ph -name '*kernel_trace.csv' | head -1); python tools/step_trace.py $f adam_multi 60 > $O/timeline_dbp_$ph.txt || exit 1
rm -rf $O/prof_$ph
head -25 $O/timeline_dbp_$ph.txt | cut -c1-150
done
