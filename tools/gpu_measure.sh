#!/usr/bin/env bash
# Measurement session: accuracy parity (native fp32 / bf16 vs reference
# expression), reference-equivalent denominators (>= 50 / 20 timed steps),
# native benches of every config.  Each step has its own time limit; stop at
# the first failure.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/measure
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
want() { for a in "${ARGS[@]}"; do [ "$a" = "$1" ] && return 0; done; return 1; }
ARGS=("$@")
if want parity; then
  timeout -k 10 900 python -u tools/parity_run.py --steps 200 \
    --out "$OUT/accuracy_parity.json" > "$OUT/parity.log" 2>&1
fi
if want ref; then
  timeout -k 10 300 python bench.py --impl reference --steps 50 --warmup 3 \
    --eval-pairs 0 --json-out "$OUT/ref_pascal.json" > "$OUT/ref_pascal.log" 2>&1
  timeout -k 10 300 python bench.py --impl reference --config willow \
    --steps 50 --warmup 3 --eval-pairs 0 --json-out "$OUT/ref_willow.json" \
    > "$OUT/ref_willow.log" 2>&1
  timeout -k 10 600 python bench.py --impl reference --config dbp15k \
    --steps 20 --warmup 2 --json-out "$OUT/ref_dbp15k.json" \
    > "$OUT/ref_dbp15k.log" 2>&1
fi
if want native; then
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 \
    --json-out "$OUT/native_pascal_fp32.json" > "$OUT/native_pascal_fp32.log" 2>&1
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --dtype bf16 \
    --json-out "$OUT/native_pascal_bf16.json" > "$OUT/native_pascal_bf16.log" 2>&1
  timeout -k 10 300 python bench.py --config willow --steps 200 --warmup 20 \
    --json-out "$OUT/native_willow_fp32.json" > "$OUT/native_willow_fp32.log" 2>&1
  timeout -k 10 600 python bench.py --config dbp15k --steps 20 --warmup 3 \
    --json-out "$OUT/native_dbp15k.json" > "$OUT/native_dbp15k.log" 2>&1
fi
echo "measure done"
