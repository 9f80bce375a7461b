#!/bin/bash
# One parameterised GPU session (replaces round 5's one-off tools/r05*_session.sh scripts):
# the steps run in order, each GPU step under its own time limit, and the session stops at
# the first failing step (fault / abort / timeout included).
#   usage: bash tools/session.sh <tag> <step> ...
#   step:  gpu=<gpu_session.sh steps, comma-separated>   e.g. gpu=tests,smoke,bench20,prof
#          env=<config>=<variant>[;<variant>...]          bench-harness A/B of the diagnostic
#                                                        library's NFN_* knobs (tools/ab_env.sh)
#          lib=<config>[,<config>...]=<checkout>[;...]    interleaved A/B of whole library builds
#                                                        under _ab/<checkout> (tools/ab_bench.sh)
#          reps=<n>                                       rounds of the A/B steps that follow (3)
# Round 5's sessions in this form, e.g. r05zv (Chain bijector rotation A/B, then the suite):
#   bash tools/session.sh r05zv 'env=bijector:C2=cur:;cur:NFN_TILE_ROT=0' gpu=tests,smoke,bench20
# and r05zr:  bash tools/session.sh r05zr gpu=tests,smoke,bench,bench20,prof,c3,c5 'env=C3=cur:;cur:NFN_TILE_ROT_G=4'
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 2
reps=3
for step in "$@"; do
  kind=${step%%=*}; arg=${step#*=}
  echo "### $TAG: $step"
  case $kind in
    gpu) bash tools/gpu_session.sh "$TAG" $(echo "$arg" | tr ',' ' ') || exit $? ;;
    env) cfg=${arg%%=*}; IFS=';' read -r -a vs <<< "${arg#*=}"
         REPS=$reps timeout -k 10 900 bash tools/ab_env.sh "${TAG}_$(echo "$cfg" | tr ':' '_')" "$cfg" "${vs[@]}" || exit $? ;;
    lib) cfgs=$(echo "${arg%%=*}" | tr ',' ' '); IFS=';' read -r -a vs <<< "${arg#*=}"
         REPS=$reps timeout -k 10 1100 bash tools/ab_bench.sh "$TAG" "$cfgs" "${vs[@]}" || exit $? ;;
    reps) reps=$arg ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
exit 0
