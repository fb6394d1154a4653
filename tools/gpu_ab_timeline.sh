# Same-box A/B of the production library against the diagnostic build
# (built from an older revision for the comparison): headline bench pairs
# and one-step kernel timelines of both.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_slot_gemm_x6.py tests/test_slot_gemm.py tests/test_dgmc.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_ab.log 2>&1 || { tail -5 gpurun_out/pt_ab.log; exit 1; }
tail -1 gpurun_out/pt_ab.log
for d in 0 1 0 1; do DGMC_AMD_DIAG=$d timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/ab_pas.log 2>&1 || exit 1; echo "pascal diag=$d $(tail -1 gpurun_out/ab_pas.log | cut -c100-190)"; done
for d in 0 1; do
  DGMC_AMD_DIAG=$d timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$d -o run -- python bench.py --steps 20 --warmup 5 > gpurun_out/prof_$d.log 2>&1 || exit 1
  f=$(find gpurun_out/prof_$d -name '*kernel_trace.csv' | head -1); python tools/step_trace.py $f > gpurun_out/timeline_diag$d.txt || exit 1
  rm -rf gpurun_out/prof_$d
done
head -12 gpurun_out/timeline_diag0.txt | cut -c1-100
# PMC pass (counters only, own run): MFMA busy share of the slot GEMMs
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc -o run -- python tools/bench_slot_gemm_x6.py --reps 2 > gpurun_out/pmc.log 2>&1 || exit 1
f=$(find gpurun_out/pmc -name '*counter_collection.csv' | head -1); python tools/pmc_summary.py $f slot_gemm_x6 > gpurun_out/pmc_x6.txt || exit 1
rm -rf gpurun_out/pmc
