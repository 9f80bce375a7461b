#!/bin/bash
# Round 5: rotated tile slots in the C2 backward (diag NFN_TILE_ROT_B): bitwise check, A/B.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r05zx
timeout -k 10 120 python tools/grad_rot_check.py > gpurun_out/r05zx/grad_rot_check.log 2>&1 || { tail -20 gpurun_out/r05zx/grad_rot_check.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zx/grad_rot_check.log
REPS=3 timeout -k 10 500 bash tools/ab_env.sh r05zx grad:C2 cur: cur:NFN_TILE_ROT_B=4 || exit $?
