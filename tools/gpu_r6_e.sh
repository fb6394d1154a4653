#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_tn.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -u tools/bench_gemm_tn.py --cfgs 0 3 --json $O/bench_tn.json > $O/bench_tn.log 2>&1 || { tail -20 $O/bench_tn.log; exit 1; }
cat $O/bench_tn.log
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d $O/pmc3 -o run -- python tools/bench_gemm_tn.py --only relconv_l12_dW --cfgs 3 --no-torch --reps 3 > $O/pmc3.log 2>&1 || { tail -5 $O/pmc3.log; exit 1; }
f=$(find $O/pmc3 -name '*counter_collection.csv' | head -1); python tools/pmc_summary.py $f gemm_tn > $O/pmc_tn_cfg3.txt; rm -rf $O/pmc3
cat $O/pmc_tn_cfg3.txt | cut -c1-300
