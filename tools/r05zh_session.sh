#!/bin/bash
# Round 5: where bench.py's ~6 us per step between kernels comes from (the legacy default
# stream?): tools/graph_gap.py, then the bench on its own stream (this tree) vs the default
# stream (HEAD~ form, via --event-mode only: both record dispatch events).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r05zh
mkdir -p $O
timeout -k 10 200 python tools/graph_gap.py 100 > $O/graph_gap.log 2>&1 || { tail -5 $O/graph_gap.log; exit 1; }
grep -v amdgpu.ids $O/graph_gap.log
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python - $O/$tag.json $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
print(sys.argv[2], "kernel %.4f step %.4f value %.4g" % (d["roofline"]["kernel_ms"], d["ms_per_step"], d["value"]))
PY
}
for r in 1 2 3; do
  run c2_dispatch_$r
  run c2_marker_$r --event-mode marker
done
for c in C5 C3; do
  run ${c}_$c --config $c
done
run C2_grad --mode grad
run C2_grid --mode grid
