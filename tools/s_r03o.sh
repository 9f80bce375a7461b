set -o pipefail
mkdir -p gpurun_out/r03o
timeout -k 10 200 python bench.py > gpurun_out/r03o/bench_default.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r03o/bench_default2.log 2>&1 && \
bash tools/gpu_session.sh r03o prof c5
