set -o pipefail
O=gpurun_out/r03k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python tools/grid_ab.py > $O/grid_ab.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --mode grid --steps 20 --warmup 5 > $O/bench_grid.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --mode grid --config C3 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_grid_c3.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_grid -o p -- python3 bench.py --mode grid --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_grid.log 2>&1
