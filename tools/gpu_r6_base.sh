#!/usr/bin/env bash
# Round-6 baseline on a fresh box: headline bench, DBP15K bench (both
# phases) and a one-step kernel timeline of DBP15K phase 1 (psi_1 trained,
# num_steps=0: /root/reference/examples/dbp15k.py:64-66).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6base; mkdir -p $O
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > $O/pascal.log 2>&1 || { tail -20 $O/pascal.log; exit 1; }
tail -1 $O/pascal.log | cut -c1-200
timeout -k 10 300 python bench.py --config dbp15k --steps 20 --warmup 3 > $O/dbp.log 2>&1 || { tail -20 $O/dbp.log; exit 1; }
tail -1 $O/dbp.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_p1 -o run -- python bench.py --config dbp15k --kg-phase phase1 --steps 5 --warmup 2 > $O/prof_p1.log 2>&1 || { tail -20 $O/prof_p1.log; exit 1; }
f=$(find $O/prof_p1 -name '*kernel_trace.csv' | head -1); python tools/step_trace.py $f adam_multi 60 > $O/timeline_dbp_p1.txt || exit 1
rm -rf $O/prof_p1
head -40 $O/timeline_dbp_p1.txt | cut -c1-150
