set -euo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
rm -f gpurun_out/bsg.log
for r in 8 12 16; do
  echo "== rounds $r" >> gpurun_out/bsg.log
  DGMC_WG_ROUNDS_1024=$r timeout -k 10 200 python tools/bench_slot_gemm.py --reps 20 --only 1024 >> gpurun_out/bsg.log 2>&1
done
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/bench_fp32.log 2>&1
echo ok
