set -o pipefail
mkdir -p gpurun_out/ab
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench.py --steps 200 --warmup 5 > gpurun_out/ab/tuned.log 2>&1 && tail -1 gpurun_out/ab/tuned.log | cut -c1-200 &&
DGMC_AMD_TUNED_GEMMS=0 timeout -k 10 300 python bench.py --steps 200 --warmup 5 > gpurun_out/ab/untuned.log 2>&1 && tail -1 gpurun_out/ab/untuned.log | cut -c1-200 &&
timeout -k 10 300 python bench.py --config willow --steps 100 --warmup 5 > gpurun_out/ab/willow.log 2>&1 && tail -1 gpurun_out/ab/willow.log | cut -c1-200 &&
timeout -k 10 300 python bench.py --config dbp15k --steps 20 --warmup 3 > gpurun_out/ab/dbp.log 2>&1 && tail -1 gpurun_out/ab/dbp.log | cut -c1-300 &&
DGMC_AMD_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/ab/gloo2.log 2>&1 && tail -1 gpurun_out/ab/gloo2.log | cut -c1-250
