#!/bin/bash
# Round 5: kernel events recorded by the launch itself (nfn_set_launch_events, hipExtLaunchKernel)
# vs hipEventRecord markers around every step, in the release bench: interleaved, every mode
# whose step is one dominant launch.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r05zf
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_launch_events.py tests/test_c_abi.py -x -v --timeout 120 \
  --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python - $O/$tag.json $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
print(sys.argv[2], "kernel %.4f step %.4f value %.4g" % (d["roofline"]["kernel_ms"], d["ms_per_step"], d["value"]), d.get("kernel_events"))
PY
}
for r in 1 2 3; do
  run c2_marker_$r --event-mode marker
  run c2_dispatch_$r --event-mode dispatch
done
for m in "C5:forward" "C3:forward" "C2:grad" "C2:dense" "C2:bijector" "C2:grid" "C2:dense_grad"; do
  c=${m%%:*}; mode=${m#*:}
  for r in 1 2; do
    run ${c}_${mode}_marker_$r --config $c --mode $mode --event-mode marker
    run ${c}_${mode}_dispatch_$r --config $c --mode $mode --event-mode dispatch
  done
done
