set -o pipefail
mkdir -p gpurun_out/r03r
timeout -k 10 300 python -u tools/microbench.py gradab 2>&1 | grep -v amdgpu.ids > gpurun_out/r03r/gradab.log && \
timeout -k 10 200 python bench.py --mode flows --flow-params separate --steps 20 --warmup 5 --cpu-seconds 6 > gpurun_out/r03r/bench_flows_separate.log 2>&1 && \
timeout -k 10 200 python bench.py --mode flows --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03r/bench_flows_views.log 2>&1
