set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/fin
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/fin/pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/fin/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.log 2>&1 || exit 1
echo smoke ok
for c in pascal willow dbp15k; do timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 10 --json-out gpurun_out/fin/bench_$c.json > gpurun_out/fin/bench_$c.log 2>&1 || exit 1; echo "$c $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fin/bench_$c.json)"; done
timeout -k 10 300 python bench.py --normalization sinkhorn --steps 100 --warmup 10 --json-out gpurun_out/fin/bench_sinkhorn.json > gpurun_out/fin/bench_sink.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --dtype bf16 --steps 100 --warmup 10 --json-out gpurun_out/fin/bench_bf16.json > gpurun_out/fin/bench_bf16.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/fin/bench_default.log 2>&1 || exit 1
echo "sinkhorn $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fin/bench_sinkhorn.json) bf16 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fin/bench_bf16.json) default $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fin/bench_default.log)"


