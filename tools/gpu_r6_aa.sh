#!/usr/bin/env bash
# A/B on the diagnostic build: rows per lane group of the ELL rowmap SpMM
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6aa; mkdir -p $O
for r in 2 4 2 4; do
  DGMC_AMD_DIAG=1 DGMC_ROWMAP_RPL=$r timeout -k 10 300 python bench.py --steps 100 --warmup 10 > $O/b_$r.log 2>&1 || { tail -5 $O/b_$r.log; exit 1; }
  echo "rpl=$r $(tail -1 $O/b_$r.log | cut -c60-140)"
done
