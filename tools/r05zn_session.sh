#!/bin/bash
# Round 5: XCD-rotated tile slots in the C2 stream (diag NFN_TILE_ROT): wave end-time spread
# (tools/wave_tail.py) and the bench-harness A/B.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r05zn
mkdir -p $O
for r in 0 4 1 12; do
  NFN_TILE_ROT=$r timeout -k 10 120 python tools/wave_tail.py C2 2 > $O/wave_tail_rot$r.log 2>&1 || { tail -5 $O/wave_tail_rot$r.log; exit 1; }
  grep -v amdgpu.ids $O/wave_tail_rot$r.log
done
REPS=3 timeout -k 10 500 bash tools/ab_env.sh r05zn C2 cur: cur:NFN_TILE_ROT=4 cur:NFN_TILE_ROT=1 cur:NFN_TILE_ROT=12 || exit $?
