#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6u; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d $O/p1 -o run -- python tools/micro/bench_dense_nt.py > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
f=$(find $O/p1 -name '*counter_collection.csv' | head -1); python tools/pmc_summary.py $f dense_nt_x6 > $O/pmc1.txt || exit 1
rm -rf $O/p1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC --output-format csv -d $O/p2 -o run -- python tools/micro/bench_dense_nt.py > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
f=$(find $O/p2 -name '*counter_collection.csv' | head -1); python tools/pmc_summary.py $f dense_nt_x6 > $O/pmc2.txt || exit 1
rm -rf $O/p2
cat $O/pmc1.txt $O/pmc2.txt | cut -c1-600
