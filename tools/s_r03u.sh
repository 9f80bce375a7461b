set -o pipefail
mkdir -p gpurun_out/r03u
for r in 1 2 3; do
  for e in 4 1; do
    timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --event-every $e > gpurun_out/r03u/c2_e${e}_$r.log 2>&1 || exit $?
    timeout -k 10 200 python bench.py --config C5 --steps 50 --warmup 10 --no-cpu-baseline --event-every $e > gpurun_out/r03u/c5_e${e}_$r.log 2>&1 || exit $?
  done
done
