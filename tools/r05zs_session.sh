#!/bin/bash
# Round 5: the C2 stream's last steps split 3 : 1 between even- and odd-XCD waves (diag
# NFN_XCD_SKEW = L steps): bitwise check, wave end times, bench-harness A/B.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r05zs
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_diag.py -x -v --timeout 200 -k strategies > $O/diag_test.log 2>&1 || { tail -30 $O/diag_test.log; exit 1; }
tail -2 $O/diag_test.log
NFN_XCD_SKEW=6 timeout -k 10 120 python tools/wave_tail.py C2 2 > $O/wave_tail_skew6.log 2>&1 || { tail -5 $O/wave_tail_skew6.log; exit 1; }
grep -v amdgpu.ids $O/wave_tail_skew6.log
REPS=3 timeout -k 10 500 bash tools/ab_env.sh r05zs C2 cur: cur:NFN_XCD_SKEW=4 cur:NFN_XCD_SKEW=6 cur:NFN_XCD_SKEW=8 || exit $?
