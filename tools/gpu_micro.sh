set -euo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/prof_quick.sh prof_sink --normalization sinkhorn > gpurun_out/prof_sink_head.txt 2>&1
head -30 gpurun_out/prof_sink_head.txt
