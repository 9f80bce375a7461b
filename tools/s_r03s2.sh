set -o pipefail
mkdir -p gpurun_out/r03s2
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "split or bijector or flow" > gpurun_out/r03s2/tests.log 2>&1 || exit $?
for m in views separate strided; do
  timeout -k 10 200 python bench.py --mode flows --flow-params $m --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03s2/bench_flows_$m.log 2>&1 || exit $?
done
