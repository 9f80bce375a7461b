set -o pipefail
O=gpurun_out/r03j
mkdir -p $O
for m in separate strided; do
  timeout -k 10 200 python bench.py --mode flows --config C3 --flow-params $m --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_flows_c3_$m.log 2>&1 || exit $?
done
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --steps 50 --warmup 10 > $O/bench.log 2>&1
