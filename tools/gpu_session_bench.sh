set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in pascal willow dbp15k; do timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 10 > gpurun_out/bench_$c.log 2>&1 || exit 1; echo "$c $(tail -1 gpurun_out/bench_$c.log | cut -c100-200)"; done
timeout -k 10 300 python bench.py --normalization sinkhorn --steps 100 --warmup 10 > gpurun_out/bench_sink.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --dtype bf16 --steps 100 --warmup 10 > gpurun_out/bench_bf16.log 2>&1 || exit 1
echo "sink/bf16 done"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_p -o run -- python bench.py --steps 20 --warmup 5 > gpurun_out/prof_p.log 2>&1 || exit 1
f=$(find gpurun_out/prof_p -name '*kernel_trace.csv' | head -1); python tools/step_trace.py $f > gpurun_out/timeline_pascal.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_d -o run -- python bench.py --config dbp15k --steps 20 --warmup 5 > gpurun_out/prof_d.log 2>&1 || exit 1
f=$(find gpurun_out/prof_d -name '*kernel_trace.csv' | head -1); python tools/step_trace.py $f > gpurun_out/timeline_dbp.txt || exit 1
head -3 gpurun_out/timeline_pascal.txt gpurun_out/timeline_dbp.txt
rm -rf gpurun_out/prof_p gpurun_out/prof_d
