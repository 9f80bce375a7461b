#!/bin/bash
# Round 5: log_prob store cache policy (nt vs sc1) x chain form across the forward lines.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
REPS=3 timeout -k 10 300 bash tools/ab_env.sh r05w_c2 C2 cur: cur:NFN_STORE_AUX=16 cur:NFN_CHAIN_FORM=8 \
  cur:NFN_CHAIN_FORM=8,NFN_STORE_AUX=16 || exit $?
REPS=2 timeout -k 10 200 bash tools/ab_env.sh r05w_c5 C5 cur: cur:NFN_STORE_AUX=16 || exit $?
REPS=2 timeout -k 10 200 bash tools/ab_env.sh r05w_c3 C3 cur: cur:NFN_STORE_AUX=16 || exit $?
REPS=2 timeout -k 10 200 bash tools/ab_env.sh r05w_r10 R10 cur: cur:NFN_STORE_AUX=16 cur:NFN_CHAIN_FORM=8 \
  cur:NFN_CHAIN_FORM=8,NFN_STORE_AUX=16 || exit $?
timeout -k 10 120 ./tools/mixed_stream > gpurun_out/r05w_mixed_stream.log 2>&1 || exit $?
cat gpurun_out/r05w_mixed_stream.log
