#!/usr/bin/env bash
# PascalVOC step timeline (aggregated and launch sequence).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6l; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --steps 5 --warmup 2 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1); python tools/step_trace.py $f adam_multi 80 > $O/timeline.txt && python tools/step_trace.py $f adam_multi 400 --seq > $O/seq.txt || exit 1
rm -rf $O/prof
head -45 $O/timeline.txt | cut -c1-150
