set -euo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_slot_gemm.py tests/test_hip_kernels.py tests/test_determinism.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/t_sg.log 2>&1
timeout -k 10 200 python tools/bench_slot_gemm.py --reps 20 > gpurun_out/bsg.log 2>&1
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/bench_fp32.log 2>&1
echo ok
