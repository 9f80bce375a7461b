set -o pipefail
mkdir -p gpurun_out/r03p
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread 2>&1 | grep -v amdgpu.ids > gpurun_out/r03p/pytest_gpu.log && \
timeout -k 10 200 python bench.py > gpurun_out/r03p/bench.log 2>&1 && \
timeout -k 10 200 python bench.py --config C5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03p/bench_c5.log 2>&1
