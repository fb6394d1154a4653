set -euo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/head
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --json-out $OUT/pascal.json > $OUT/pascal.log 2>&1
tail -1 $OUT/pascal.log | cut -c1-200
