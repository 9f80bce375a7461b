set -o pipefail
bash tools/gpu_session.sh r03h testsx smoke bench prof c5 prof_c5 c3 grad prof_grad grad_c3 dense dense_c5 dgrad bijector || exit $?
for m in views separate strided; do
  timeout -k 10 200 python bench.py --mode flows --flow-params $m --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03h/bench_flows_$m.log 2>&1 || exit $?
done
