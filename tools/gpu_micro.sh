set -euo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/ex
mkdir -p $OUT
timeout -k 10 600 python -u examples/pascal.py --epochs 15 > $OUT/pascal.log 2>&1
tail -8 $OUT/pascal.log
timeout -k 10 600 python -u examples/willow.py --runs 3 > $OUT/willow.log 2>&1
tail -6 $OUT/willow.log
