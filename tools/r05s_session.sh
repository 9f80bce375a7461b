#!/bin/bash
# Round 5: the C2 forward's structure vs a pure stream on one box (tools/stream_ceiling.hip),
# then the bench-harness knob sweeps of the other lines.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r05s
timeout -k 10 120 ./tools/stream_ceiling > gpurun_out/r05s/stream_ceiling.log 2>&1 || exit $?
cat gpurun_out/r05s/stream_ceiling.log
REPS=2 timeout -k 10 200 bash tools/ab_env.sh r05s C2 cur: cur:NFN_ABLATE_FLOWS=1 || exit $?
bash tools/r05r_session.sh
