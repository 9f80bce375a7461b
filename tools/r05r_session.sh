#!/bin/bash
# Round 5: bench-harness knob sweeps of the other forward / backward lines (diag library).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
REPS=2 timeout -k 10 300 bash tools/ab_env.sh r05r_c3 C3 cur: cur:NFN_WG_PER_CU=1 cur:NFN_WG_PER_CU=3 cur:NFN_PRIO=0 \
  cur:NFN_ABLATE_FLOWS=1 cur:NFN_ABLATE_LOADS=1 || exit $?
REPS=2 timeout -k 10 300 bash tools/ab_env.sh r05r_c5 C5 cur: cur:NFN_WG_PER_CU=1 cur:NFN_WG_PER_CU=3 cur:NFN_WG_PER_CU=4 \
  cur:NFN_CHAIN_FORM=3 cur:NFN_ABLATE_FLOWS=1 cur:NFN_ABLATE_LOADS=1 || exit $?
REPS=2 timeout -k 10 300 bash tools/ab_env.sh r05r_grad grad:C2 cur: cur:NFN_ABLATE_FLOWS=1 cur:NFN_ABLATE_LOADS=1 \
  cur:NFN_GRAD_WPB=1 cur:NFN_GRAD_WPB=4 || exit $?
