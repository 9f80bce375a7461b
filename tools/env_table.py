"""One line per run of a tools/ab_env.sh tag (the bench harness's diagnostic-library A/B):
name, repetition, kernel ms, step ms, config and the NFN_* knobs it ran with.

  python tools/env_table.py gpurun_out/<tag> > profiles/<round>/<tag>_bench_diag.txt"""

import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    tag = os.path.basename(os.path.normpath(d))
    print(f"# tools/ab_env.sh {tag} (bench.py --diag, diagnostic libraries): name rep kernel_ms step_ms config env")
    rows = []
    for f in glob.glob(os.path.join(d, "*.json")):
        name, rep = os.path.basename(f)[:-5].rsplit("_", 1)
        lines = [ln for ln in open(f) if ln.startswith("{")]
        if not lines:
            continue
        j = json.loads(lines[0])
        env = j.get("nfn_env", j.get("env", {}))
        rows.append((int(rep), os.path.getmtime(f), name, j["roofline"]["kernel_ms"], j["ms_per_step"],
                     j["config"].get("workload", "")[:3], env))
    for rep, _, name, k, st, cfg, env in sorted(rows, key=lambda r: r[1]):
        print(f"{name} {rep} {k:.4f} {st:.4f} {cfg} {env}")


if __name__ == "__main__":
    main()
