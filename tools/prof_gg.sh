#!/usr/bin/env bash
# rocprofv3 kernel durations of tools/bench_gg.py under DGMC_GG_DEBUG modes.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONPATH=$PWD
OUT=$PWD/gpurun_out/gg
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for m in 0 1 2 3; do
  DGMC_GG_DEBUG=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/m$m -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_gg.py > $OUT/m$m.log 2>&1
done
