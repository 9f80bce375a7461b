#!/bin/bash
# Interleaved A/B of whole library builds on one box: each variant is a checkout under
# _ab/<name>/ with its own in-tree libnfn_hip.so and bench.py ("cur" = this tree).
#   usage: bash tools/ab_bench.sh <tag> "<configs>" <variants...>
# A config token is CONFIG or MODE:CONFIG (e.g. "C2 C5 grad:C2 dense:C2").
set -o pipefail
TAG=$1; CFGS=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
for r in $(seq 1 ${REPS:-3}); do
  for cfg in $CFGS; do
    for v in "$@"; do
      dir=$ROOT/_ab/$v; [ "$v" = cur ] && dir=$ROOT
      mode=forward; c=$cfg
      case $cfg in *:*) mode=${cfg%%:*}; c=${cfg#*:};; esac
      timeout -k 10 120 python "$dir/bench.py" --mode $mode --config $c --steps 50 --warmup 10 --no-cpu-baseline \
        > "$OUT/${cfg}_${v}_$r.json" 2> "$OUT/${cfg}_${v}_$r.err"
      rc=$?
      echo "$cfg $v $r rc=$rc $(python -c "import json,sys; d=json.loads([l for l in open('$OUT/${cfg}_${v}_$r.json') if l.startswith('{')][0]); print(round(d['roofline']['kernel_ms'],4), round(d['ms_per_step'],4))" 2>/dev/null)"
      if [ $rc -ne 0 ]; then exit $rc; fi
    done
  done
done
exit 0
