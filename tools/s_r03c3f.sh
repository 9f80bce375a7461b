set -o pipefail
mkdir -p gpurun_out/r03c3f
for m in views separate strided; do
  timeout -k 10 200 python bench.py --mode flows --config C3 --flow-params $m --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03c3f/bench_flows_c3_$m.log 2>&1 || exit $?
done
timeout -k 10 200 python bench.py --mode bijector --config C3 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03c3f/bench_bijector_c3.log 2>&1
