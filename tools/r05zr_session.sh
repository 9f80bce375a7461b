#!/bin/bash
# Round 5: the library with rotated tile slots by default (chain_wave1_kernel): GPU suite, smoke,
# bench lines, rocprof; then the C3 lane-group kernel's rotation A/B (diag NFN_TILE_ROT_G).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/gpu_session.sh r05zr tests smoke bench bench20 prof c3 c5 || exit $?
REPS=3 timeout -k 10 400 bash tools/ab_env.sh r05zr_c3 C3 cur: cur:NFN_TILE_ROT_G=4 || exit $?
