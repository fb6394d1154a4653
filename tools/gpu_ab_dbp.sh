# Same-box A/B on the DBP15K refinement step: production library vs the
# diagnostic build of an older revision; tests first, then bench pairs and
# one-step kernel timelines of both.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gemm_f32.py tests/test_relconv.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_ab.log 2>&1 || { tail -5 gpurun_out/pt_ab.log; exit 1; }
tail -1 gpurun_out/pt_ab.log
for d in 0 1 0 1; do DGMC_AMD_DIAG=$d timeout -k 10 300 python bench.py --config dbp15k --steps 50 --warmup 10 > gpurun_out/ab_dbp.log 2>&1 || exit 1; echo "dbp diag=$d $(tail -1 gpurun_out/ab_dbp.log | cut -c150-230)"; done
for d in 0 1; do
  DGMC_AMD_DIAG=$d timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$d -o run -- python bench.py --config dbp15k --steps 20 --warmup 5 > gpurun_out/prof_$d.log 2>&1 || exit 1
  f=$(find gpurun_out/prof_$d -name '*kernel_trace.csv' | head -1); python tools/step_trace.py $f > gpurun_out/timeline_dbp_diag$d.txt || exit 1
  rm -rf gpurun_out/prof_$d
done
grep "step span\|gemm_nt" gpurun_out/timeline_dbp_diag0.txt gpurun_out/timeline_dbp_diag1.txt | cut -c1-140
