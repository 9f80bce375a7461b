#!/bin/bash
# Round-5 studies in the bench harness (diag library): busy-VALU pacing of the C2 forward,
# and the fused Dense kernels' compute-only / memory-only times.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
REPS=2 timeout -k 10 500 bash tools/ab_env.sh r05h C2 cur: cur:NFN_PACE=-2 cur:NFN_PACE=-4 cur:NFN_PACE=-8 cur:NFN_PACE=-12 \
  cur:NFN_PACE=-16 cur:NFN_PACE=-24 cur:NFN_ABLATE_FLOWS=1,NFN_PACE=-8 cur:NFN_ABLATE_FLOWS=1,NFN_PACE=-16 r03: || exit $?
REPS=2 timeout -k 10 300 bash tools/ab_env.sh r05i dense:C2 cur: cur:NFN_ABLATE_FLOWS=1 cur:NFN_ABLATE_LOADS=1 || exit $?
REPS=2 timeout -k 10 300 bash tools/ab_env.sh r05j dense_grad:C2 cur: cur:NFN_ABLATE_FLOWS=1 cur:NFN_ABLATE_LOADS=1 || exit $?
