set -euo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/sw
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_hip_kernels.py -k "headline_widths" > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
tail -4 $OUT/t.log
