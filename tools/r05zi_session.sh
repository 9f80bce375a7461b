#!/bin/bash
# Round 5: the wall-clock cost of timing a step with events (dispatch-recorded or markers):
# C2 bench at the driver's --steps 20 --warmup 5 with events on every E-th step.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r05zi
mkdir -p $O
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 5 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python - $O/$tag.json $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
r = d["roofline"]
print(sys.argv[2], "kernel %.4f (%d launches) step %.4f value %.4g" % (r["kernel_ms"], r["kernel_ms_launches"], d["ms_per_step"], d["value"]))
PY
}
for r in 1 2 3; do
  for e in 1 2 4 20; do
    run c2_dispatch_e${e}_$r --event-every $e
  done
  run c2_marker_e4_$r --event-mode marker --event-every 4
done
