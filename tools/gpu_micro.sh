set -euo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/s3
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --normalization sinkhorn --steps 100 --warmup 10 --json-out $OUT/sinkhorn.json > $OUT/sinkhorn.log 2>&1
tail -1 $OUT/sinkhorn.log | cut -c1-250
bash tools/prof_quick.sh prof_fp32 > $OUT/prof.txt 2>&1
head -3 $OUT/prof.txt
