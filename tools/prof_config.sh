#!/usr/bin/env bash
# rocprofv3 kernel stats of one bench config:  tools/prof_config.sh <config> [steps]
set -e
cd "${GRAFT_REPO_ROOT:-.}"
CFG=${1:-dbp15k}; STEPS=${2:-5}
OUT=$PWD/gpurun_out/prof_$CFG
rm -rf "$OUT"; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --config "$CFG" --steps "$STEPS" --warmup 2 > "$OUT/log.txt" 2>&1
tail -n 1 "$OUT/log.txt"
