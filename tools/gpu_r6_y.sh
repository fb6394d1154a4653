#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6y; mkdir -p $O
timeout -k 10 300 python -u tools/micro/relcnn_reserve_check.py > $O/res.log 2>&1 || { tail -20 $O/res.log; exit 1; }
tail -14 $O/res.log
