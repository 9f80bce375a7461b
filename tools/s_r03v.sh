set -o pipefail
mkdir -p gpurun_out/r03v
timeout -k 10 300 python -u tools/microbench.py fwdab 2>&1 | grep -v amdgpu.ids > gpurun_out/r03v/fwdab.log
