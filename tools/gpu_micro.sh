set -euo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/c2
mkdir -p $OUT
timeout -k 10 300 python tools/bench_slot_gemm.py --reps 20 --only 128 > $OUT/micro.txt 2>&1 || { tail -20 $OUT/micro.txt; exit 1; }
grep -E "rowmap" $OUT/micro.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_slot_gemm.py tests/test_hip_kernels.py tests/test_determinism.py tests/test_dp_step.py > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --json-out $OUT/b.json > $OUT/b.log 2>&1
tail -1 $OUT/b.log | cut -c1-200
