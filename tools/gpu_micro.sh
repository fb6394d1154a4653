set -euo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/csc
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_candidates.py tests/test_kg_trainer.py tests/test_hip_kernels.py > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
tail -3 $OUT/t.log
timeout -k 10 600 python bench.py --config dbp15k --steps 20 --warmup 3 > $OUT/dbp.log 2>&1
tail -1 $OUT/dbp.log | cut -c1-300
timeout -k 10 300 python bench.py --config willow --steps 200 --warmup 20 --json-out $OUT/willow.json > $OUT/willow.log 2>&1
tail -1 $OUT/willow.log | cut -c1-200
