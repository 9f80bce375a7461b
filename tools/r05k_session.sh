#!/bin/bash
# Effective engine clock (GRBM_GUI_ACTIVE / 8 / kernel time) of the C2 forward: the round-3
# library vs HEAD, full and memory-only (diag build), one rocprofv3 --pmc pass each.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp
export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/r05k
mkdir -p $OUT
pmc() {  # pmc <name> <bench dir> [--diag] ; env from the caller
  local name=$1 dir=$2; shift 2
  timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $OUT/$name -o p -- \
    python3 $dir/bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
pmc r03_full $ROOT/_ab/r03 || exit $?
pmc cur_full $ROOT || exit $?
NFN_ABLATE_FLOWS=1 pmc r03_mem $ROOT/_ab/r03 --diag || exit $?
NFN_ABLATE_FLOWS=1 pmc cur_mem $ROOT --diag || exit $?
pmc r03_full_b $ROOT/_ab/r03 || exit $?
pmc cur_full_b $ROOT || exit $?
