#!/bin/bash
# Round 5: rotated tile slots for the Chain bijector's wave1 walk too: bench-harness A/B, then the
# final library's GPU suite, smoke and bench line.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
REPS=3 timeout -k 10 400 bash tools/ab_env.sh r05zv bijector:C2 cur: cur:NFN_TILE_ROT=0 || exit $?
bash tools/gpu_session.sh r05zv tests smoke bench20 || exit $?
