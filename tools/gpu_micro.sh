set -euo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/sched
mkdir -p $OUT
timeout -k 10 300 python -m pytest -q -x tests/test_slot_gemm.py -m gpu > $OUT/t.txt 2>&1 || { tail -30 $OUT/t.txt; exit 1; }
tail -1 $OUT/t.txt
timeout -k 10 300 python tools/bench_slot_gemm.py --reps 20 > $OUT/v2.txt 2>&1
grep -E "fwd2|dX2|wgrad" $OUT/v2.txt
