#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6t; mkdir -p $O
timeout -k 10 300 python -u tools/micro/bench_dense_nt.py > $O/nt.log 2>&1 || { tail -20 $O/nt.log; exit 1; }
cat $O/nt.log
