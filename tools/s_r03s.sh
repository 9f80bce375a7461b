set -o pipefail
mkdir -p gpurun_out/r03s
timeout -k 10 300 python -u tools/microbench.py evcost 2>&1 | grep -v amdgpu.ids > gpurun_out/r03s/evcost.log
