set -o pipefail
bash tools/gpu_session.sh r03f testsx smoke bench prof c5 prof_c5 c3 grad prof_grad grad_c3 dense dense_c5 dgrad bijector || exit $?
mkdir -p gpurun_out/r03f
timeout -k 10 200 python bench.py --mode flows --steps 10 --warmup 3 --cpu-seconds 6 > gpurun_out/r03f/bench_flows_views.log 2>&1 && \
timeout -k 10 200 python bench.py --mode flows --flow-params separate --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03f/bench_flows_separate.log 2>&1
