set -o pipefail
mkdir -p gpurun_out/r03g
timeout -k 10 300 python tools/microbench.py dma > gpurun_out/r03g/dma_ab.log 2>&1; echo "dma rc=$?"
cat gpurun_out/r03g/dma_ab.log | grep -v amdgpu.ids | cut -c1-200
timeout -k 10 120 python bench.py --mode flows --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03g/bench_flows.log 2>&1; echo "flows rc=$?"
tail -1 gpurun_out/r03g/bench_flows.log | cut -c1-400
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "bijector or single_flow or reference_flow" > gpurun_out/r03g/pytest_flows.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/r03g/pytest_flows.log
