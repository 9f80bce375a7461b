#!/bin/bash
# Round 5: the next tile's rows issued in two halves (diag NFN_SPLIT_ISSUE=1), the second after
# half of the pair bodies (tools/inflight_probe.hip: a C2-shaped stream with the chain's VALU
# time ran 0.348 vs 0.381 ms that way), bitwise check, then the bench-harness A/B.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r05zd
timeout -k 10 200 python -u -m pytest tests/test_gpu_diag.py -x -v --timeout 200 -k strategies > gpurun_out/r05zd/diag_test.log 2>&1 || { tail -30 gpurun_out/r05zd/diag_test.log; exit 1; }
tail -3 gpurun_out/r05zd/diag_test.log
REPS=4 timeout -k 10 500 bash tools/ab_env.sh r05zd C2 cur: cur:NFN_SPLIT_ISSUE=1 || exit $?
REPS=2 timeout -k 10 300 bash tools/ab_env.sh r05zd R10 cur: cur:NFN_SPLIT_ISSUE=1 || exit $?
