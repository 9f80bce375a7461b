#!/bin/bash
# Round 5: issue order at the C2 hand-off (NFN_EARLY_ISSUE) and the kernel's memory-only form
# at one workgroup per CU, beside the pure stream on the same box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r05za
timeout -k 10 120 ./tools/stream_ceiling > gpurun_out/r05za/stream_ceiling.log 2>&1 || exit $?
head -2 gpurun_out/r05za/stream_ceiling.log
REPS=3 timeout -k 10 500 bash tools/ab_env.sh r05za C2 cur: cur:NFN_EARLY_ISSUE=1 cur:NFN_ABLATE_FLOWS=1 \
  cur:NFN_ABLATE_FLOWS=1,NFN_EARLY_ISSUE=1 cur:NFN_ABLATE_FLOWS=1,NFN_WG_PER_CU=1 cur:NFN_WG_PER_CU=1 || exit $?
