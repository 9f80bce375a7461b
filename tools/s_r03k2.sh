set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r03k2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_grid -o grid -- python3 $GRAFT_REPO_ROOT/bench.py --mode grid --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_grid.log 2>&1
