set -o pipefail
mkdir -p gpurun_out/r03n
timeout -k 10 300 python -u tools/microbench.py dgradceil 2>&1 | grep -v amdgpu.ids > gpurun_out/r03n/dgradceil.log && \
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullbatch.py -x -v -s --timeout 600 --timeout-method thread 2>&1 | grep -v amdgpu.ids > gpurun_out/r03n/fullbatch.log
