#!/bin/bash
# Interleaved A/B in the bench harness itself with the DIAGNOSTIC libraries (bench.py --diag):
# each variant is <checkout>:<NFN knobs>, e.g. "r03:NFN_ABLATE_FLOWS=1" or "cur:" ("cur" = this
# tree).  Ablation / tuning studies only (memory-only, compute-only, occupancy, chain forms).
#   usage: REPS=3 bash tools/ab_env.sh <tag> <config> <variant> ...
set -o pipefail
TAG=$1; CFG=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
mode=forward; c=$CFG
case $CFG in *:*) mode=${CFG%%:*}; c=${CFG#*:};; esac
for r in $(seq 1 ${REPS:-3}); do
  for spec in "$@"; do
    v=${spec%%:*}; knobs=${spec#*:}
    dir=$ROOT/_ab/$v; [ "$v" = cur ] && dir=$ROOT
    name=$(echo "${v}_${knobs}" | tr '=,' '-_')
    env $(echo "$knobs" | tr ',' ' ') timeout -k 10 120 python "$dir/bench.py" --diag --mode $mode --config $c --steps 50 \
      --warmup 10 --no-cpu-baseline > "$OUT/${name}_$r.json" 2> "$OUT/${name}_$r.err"
    rc=$?
    echo "$spec $r rc=$rc $(python -c "import json; d=json.loads([l for l in open('$OUT/${name}_$r.json') if l.startswith('{')][0]); print(round(d['roofline']['kernel_ms'],4), round(d['ms_per_step'],4))" 2>/dev/null)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
exit 0
