set -o pipefail
mkdir -p gpurun_out/r03l
timeout -k 10 300 python tools/microbench.py gradshape 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03l/gradshape.log | cut -c1-200
timeout -k 10 200 python tools/microbench.py flows 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03l/flows.log | cut -c1-200
timeout -k 10 700 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/r03l/pytest_gpu.log 2>&1
echo "pytest rc=$?"
tail -4 gpurun_out/r03l/pytest_gpu.log
