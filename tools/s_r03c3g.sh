set -o pipefail
mkdir -p gpurun_out/r03c3g
timeout -k 10 400 python -u -m pytest tests/test_gpu_diag.py tests/test_gpu_split.py tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "flow or diag or split or bijector or radial" > gpurun_out/r03c3g/tests.log 2>&1 || exit $?
for m in views separate strided; do
  timeout -k 10 200 python bench.py --mode flows --config C3 --flow-params $m --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03c3g/bench_flows_c3_$m.log 2>&1 || exit $?
done
timeout -k 10 200 python bench.py --mode flows --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03c3g/bench_flows_c2_views.log 2>&1
