set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r04q
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch_c2 -o f -- python3 $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/pmc_fetch_c2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write_c2 -o w -- python3 $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/pmc_write_c2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch_c5 -o f -- python3 $ROOT/bench.py --config C5 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/pmc_fetch_c5.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write_c5 -o w -- python3 $ROOT/bench.py --config C5 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/pmc_write_c5.log 2>&1
