set -euo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/os
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_candidates.py tests/test_kg_trainer.py > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 600 python bench.py --config dbp15k --steps 20 --warmup 3 --json-out $OUT/dbp.json > $OUT/dbp.log 2>&1
tail -1 $OUT/dbp.log | cut -c1-250
