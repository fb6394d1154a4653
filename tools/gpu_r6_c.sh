#!/usr/bin/env bash
# TN GEMM staging variants + PMC, top-k warm start micro-benchmark.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_tn.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -u tools/bench_gemm_tn.py --json $O/bench_tn.json > $O/bench_tn.log 2>&1 || { tail -20 $O/bench_tn.log; exit 1; }
cat $O/bench_tn.log
timeout -k 10 300 python -u tools/bench_topk_warm.py --json $O/topk_warm.json > $O/topk_warm.log 2>&1 || { tail -20 $O/topk_warm.log; exit 1; }
cat $O/topk_warm.log
for c in 0 1; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d $O/pmc$c -o run -- python tools/bench_gemm_tn.py --only relconv_l12_dW --cfgs $c --no-torch --reps 3 > $O/pmc$c.log 2>&1 || { tail -5 $O/pmc$c.log; exit 1; }
f=$(find $O/pmc$c -name '*counter_collection.csv' | head -1); python tools/pmc_summary.py $f gemm_tn > $O/pmc_tn_cfg$c.txt || exit 1
rm -rf $O/pmc$c
cat $O/pmc_tn_cfg$c.txt | cut -c1-400
done
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC --output-format csv -d $O/pmc2 -o run -- python tools/bench_gemm_tn.py --only relconv_l12_dW --cfgs 0 --no-torch --reps 3 > $O/pmc2.log 2>&1 || { tail -5 $O/pmc2.log; exit 1; }
f=$(find $O/pmc2 -name '*counter_collection.csv' | head -1); python tools/pmc_summary.py $f gemm_tn > $O/pmc_tn_insts.txt || exit 1
rm -rf $O/pmc2
cat $O/pmc_tn_insts.txt | cut -c1-400
