set -euo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/prof_quick.sh prof_fp32 > gpurun_out/prof_fp32_head.txt 2>&1
head -2 gpurun_out/prof_fp32_head.txt
grep -E "sg_scan|BFloat16|FillFunctor" gpurun_out/prof_fp32/step.txt | cut -c1-120
