set -o pipefail
mkdir -p gpurun_out/r03t
timeout -k 10 200 python bench.py > gpurun_out/r03t/bench.log 2>&1 && \
timeout -k 10 200 python bench.py --config C5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03t/bench_c5.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --event-every 1 > gpurun_out/r03t/bench_every1.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_multiproc.py tests/test_gpu_comm.py -x -v --timeout 300 --timeout-method thread 2>&1 | grep -v amdgpu.ids > gpurun_out/r03t/pytest_mp.log
