#!/bin/bash
# Round-5 C2 regression study on ONE box: the round-3 library (_ab/r03) vs HEAD, as release
# builds (tools/ab_bench.sh) and as diagnostic builds (full / memory-only / compute-only,
# tools/microbench.py fwdab), interleaved; then HEAD's chain forms and occupancy (c2form5).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=gpurun_out/r05d
mkdir -p $OUT
for rep in 1 2; do
  for v in r03 tanh cur; do
    dir=_ab/$v; [ $v = cur ] && dir=.
    timeout -k 10 300 python $dir/tools/microbench.py fwdab > $OUT/fwdab_${v}_$rep.log 2>&1
    rc=$?; echo "fwdab $v $rep rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
REPS=3 timeout -k 10 400 bash tools/ab_bench.sh r05d_ab "C2" r03 tanh cur > $OUT/ab.txt 2>&1 || exit $?
cat $OUT/ab.txt
timeout -k 10 300 python tools/microbench.py c2form5 C2 > $OUT/c2form5.log 2>&1 || exit $?
echo done
