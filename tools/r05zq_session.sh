#!/bin/bash
# Round 5: second-box check of the rotated tile slots (diag NFN_TILE_ROT=4) in the bench harness.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
REPS=4 timeout -k 10 500 bash tools/ab_env.sh r05zq C2 cur: cur:NFN_TILE_ROT=4 cur:NFN_TILE_ROT=8 || exit $?
REPS=2 timeout -k 10 300 bash tools/ab_env.sh r05zq R10 cur: cur:NFN_TILE_ROT=4 || exit $?
