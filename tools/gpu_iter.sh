set -euo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dp_step.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/t_dp.log 2>&1
echo ok
