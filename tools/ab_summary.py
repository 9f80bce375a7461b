"""Median kernel / step times per (config, variant) of a tools/ab_bench.sh run.

  python tools/ab_summary.py gpurun_out/<tag>  ->  one line per config: variant medians and
  their ratio to the first variant named on the command line (default: r3)."""

import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    base = sys.argv[2] if len(sys.argv) > 2 else "r3"
    res = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "*.json"))):
        name = os.path.basename(f)[:-5]
        cfg, var, rep = name.rsplit("_", 2)
        lines = [ln for ln in open(f) if ln.startswith("{")]
        if not lines:
            continue
        j = json.loads(lines[0])
        res[cfg][var].append((j["roofline"]["kernel_ms"], j["ms_per_step"]))
    for cfg, vs in res.items():
        b = statistics.median(k for k, _ in vs[base]) if base in vs else None
        parts = []
        for var, xs in vs.items():
            k = statistics.median(x for x, _ in xs)
            st = statistics.median(x for _, x in xs)
            rel = f" ({100 * (k / b - 1):+.1f}%)" if b else ""
            parts.append(f"{var} kernel {k:.4f} step {st:.4f}{rel} n={len(xs)}")
        print(f"{cfg}: " + "; ".join(parts))


if __name__ == "__main__":
    main()
