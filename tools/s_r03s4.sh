set -o pipefail
mkdir -p gpurun_out/r03s4
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r03s4/tests.log 2>&1 || exit $?
for m in views separate views; do
  timeout -k 10 200 python bench.py --mode flows --flow-params $m --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/r03s4/bench_flows.log 2>&1 || exit $?
done
