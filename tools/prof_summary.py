#!/usr/bin/env python3
"""Summarise rocprofv3 outputs into profiles/.

  python tools/prof_summary.py stats <rocprof_dir> <out_prefix>
      copies *_kernel_stats.csv to <out_prefix>_kernel_stats.csv and prints it
  python tools/prof_summary.py pmc <fetch_dir> <write_dir> <out_json> --cfg C2 --batch N --kernel chain_logprob
      per-launch HBM traffic of the kernel from separate FETCH_SIZE / WRITE_SIZE passes:
      bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024   (FETCH_SIZE is in KiB and on
      gfx950 reads exactly half of a wide coalesced stream: MI355X_MICROARCH.md §HBM)
"""

import argparse
import csv
import glob
import json
import os
import shutil
import statistics
import sys


def find(root, pattern):
    hits = sorted(glob.glob(os.path.join(root, "**", pattern), recursive=True))
    if not hits:
        raise SystemExit(f"no {pattern} under {root}")
    return hits


def cmd_trace(args):
    """Per-call durations of one kernel from a kernel_trace.csv: mean / median over all calls
    and over the last N (the bench's timed steps, after its prewarm and warmup)."""
    src = find(args.dir, "*kernel_trace.csv")[0]
    with open(src) as f:
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(f)
             if r["Kernel_Name"].startswith(args.kernel)]
    if not d:
        raise SystemExit(f"no {args.kernel} calls in {src}")
    last = d[-args.last:]
    rec = {"kernel": args.kernel, "calls": len(d), "mean_us": statistics.mean(d), "median_us": statistics.median(d),
           "min_us": min(d), "max_us": max(d), "last_n": len(last), "last_mean_us": statistics.mean(last),
           "last_median_us": statistics.median(last)}
    with open(args.out_json, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


def cmd_stats(args):
    src = find(args.dir, "*kernel_stats.csv")[0]
    shutil.copyfile(src, args.out_prefix + "_kernel_stats.csv")
    with open(src) as f:
        rows = list(csv.DictReader(f))
    for r in rows:
        print(f"{r['Name'][:70]:70s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs']) / 1e3:10.2f} "
              f"pct={float(r['Percentage']):6.2f}")
    # also keep the kernel trace (per-dispatch durations) for the dominant kernel
    traces = glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True)
    if traces:
        with open(traces[0]) as f:
            tr = list(csv.DictReader(f))
        durs = {}
        for r in tr:
            durs.setdefault(r["Kernel_Name"], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        summary = {k: {"calls": len(v), "avg_us": statistics.mean(v) / 1e3, "median_us": statistics.median(v) / 1e3,
                       "min_us": min(v) / 1e3, "max_us": max(v) / 1e3} for k, v in durs.items()}
        with open(args.out_prefix + "_kernel_trace_summary.json", "w") as f:
            json.dump(summary, f, indent=1)


def counter_avg(root, counter, kernel_substr):
    vals = {}
    for path in find(root, "*counter_collection.csv"):
        with open(path) as f:
            for r in csv.DictReader(f):
                if kernel_substr in r["Kernel_Name"] and r["Counter_Name"] == counter:
                    key = r.get("Dispatch_Id") or r.get("Correlation_Id")
                    vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel_substr} under {root}")
    return statistics.mean(vals.values()), len(vals)


def cmd_pmc(args):
    fetch, nf = counter_avg(args.fetch_dir, "FETCH_SIZE", args.kernel)
    write, nw = counter_avg(args.write_dir, "WRITE_SIZE", args.kernel)
    rec = {
        "config": args.cfg,
        "batch": args.batch,
        "kernel": args.kernel,
        "fetch_size_kib_raw": fetch,
        "write_size_kib": write,
        "dispatches": [nf, nw],
        "hbm_bytes_per_launch": 2.0 * fetch * 1024.0 + write * 1024.0,
        "correction": "FETCH_SIZE x2 (gfx950 reports half of a 16B/lane coalesced stream), KiB -> bytes",
        "algorithmic_bytes_per_launch": args.alg_bytes,
    }
    if args.alg_bytes:
        rec["traffic_over_algorithmic"] = rec["hbm_bytes_per_launch"] / args.alg_bytes
    with open(args.out_json, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("stats")
    s.add_argument("dir")
    s.add_argument("out_prefix")
    tr = sub.add_parser("trace")
    tr.add_argument("dir")
    tr.add_argument("out_json")
    tr.add_argument("--kernel", default="chain_wave1_kernel")
    tr.add_argument("--last", type=int, default=50)
    tr.set_defaults(fn=cmd_trace)
    p = sub.add_parser("pmc")
    p.add_argument("fetch_dir")
    p.add_argument("write_dir")
    p.add_argument("out_json")
    p.add_argument("--cfg", default="C2")
    p.add_argument("--batch", type=int, default=1 << 24)
    p.add_argument("--kernel", default="chain_logprob")
    p.add_argument("--alg-bytes", type=float, default=None)
    args = ap.parse_args()
    {"stats": cmd_stats, "pmc": cmd_pmc, "trace": cmd_trace}[args.cmd](args)


if __name__ == "__main__":
    sys.exit(main())
