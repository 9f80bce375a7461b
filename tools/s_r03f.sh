set -o pipefail
mkdir -p gpurun_out/r03f
timeout -k 10 700 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/r03f/pytest_gpu.log 2>&1
echo "pytest rc=$?"
tail -8 gpurun_out/r03f/pytest_gpu.log
timeout -k 10 120 python bench.py --mode flows --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03f/bench_flows.log 2>&1 || exit $?
tail -1 gpurun_out/r03f/bench_flows.log | cut -c1-300
REPS=2 bash tools/ab_bench.sh r03f_ab "C3 grad:C2 grad:C3 dense_grad:C2 bijector:C2" base cur
