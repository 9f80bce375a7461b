set -o pipefail
mkdir -p gpurun_out/r03w
timeout -k 10 300 python -u tools/microbench.py postx2 2>&1 | grep -v amdgpu.ids > gpurun_out/r03w/postx2.log && \
timeout -k 10 300 python -u tools/microbench.py fwdab 2>&1 | grep -v amdgpu.ids > gpurun_out/r03w/fwdab.log
