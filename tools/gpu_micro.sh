set -euo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/conf
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py --config dbp15k --steps 20 --warmup 3 --json-out $OUT/dbp.json > $OUT/dbp.log 2>&1
tail -1 $OUT/dbp.log | cut -c1-250
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --json-out $OUT/pascal.json > $OUT/pascal.log 2>&1
tail -1 $OUT/pascal.log | cut -c1-250
