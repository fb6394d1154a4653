# DBP15K refinement step with the node GEMMs on bf16x6 (default) vs the
# exact-f32 chain (DGMC_AMD_X6=0), same box: tests, bench pairs, timelines.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gemm_f32.py tests/test_relconv.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_ab.log 2>&1 || { tail -15 gpurun_out/pt_ab.log; exit 1; }
tail -1 gpurun_out/pt_ab.log
for x in 1 0 1 0; do DGMC_AMD_X6=$x timeout -k 10 300 python bench.py --config dbp15k --steps 50 --warmup 10 > gpurun_out/ab_dbp.log 2>&1 || exit 1; echo "dbp x6=$x $(tail -1 gpurun_out/ab_dbp.log | cut -c150-230) $(tail -1 gpurun_out/ab_dbp.log | grep -o '"hits@1_test": [0-9.]*')"; done
for x in 1 0; do
  DGMC_AMD_X6=$x timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$x -o run -- python bench.py --config dbp15k --steps 20 --warmup 5 > gpurun_out/prof_$x.log 2>&1 || exit 1
  f=$(find gpurun_out/prof_$x -name '*kernel_trace.csv' | head -1); python tools/step_trace.py $f > gpurun_out/timeline_dbp_x6$x.txt || exit 1
  rm -rf gpurun_out/prof_$x
done
grep "step span\|gemm_nt" gpurun_out/timeline_dbp_x61.txt gpurun_out/timeline_dbp_x60.txt | cut -c1-140
