"""Effective engine clock per dispatch of one kernel from a rocprofv3 --pmc GRBM_GUI_ACTIVE
pass (counter_collection.csv): GRBM_GUI_ACTIVE / 8 XCDs / (End - Start), per
MI355X_MICROARCH.md 'DVFS give-back'.  Prints the median over the last N dispatches.

  python tools/pmc_clock.py <dir with p_counter_collection.csv> [kernel substring] [N]"""

import csv
import glob
import os
import statistics
import sys

csv.field_size_limit(1 << 30)


def main():
    d = sys.argv[1]
    ksub = sys.argv[2] if len(sys.argv) > 2 else "chain_wave1_kernel"
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    path = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
    rows = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if ksub not in r["Kernel_Name"]:
                continue
            key = int(r["Dispatch_Id"])
            e = rows.setdefault(key, {"t": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9})
            e[r["Counter_Name"]] = float(r["Counter_Value"])
    keys = sorted(rows)[-n:]
    ghz = [rows[k]["GRBM_GUI_ACTIVE"] / 8 / rows[k]["t"] / 1e9 for k in keys]
    ms = [rows[k]["t"] * 1e3 for k in keys]
    print(f"{d}: {len(keys)} dispatches of *{ksub}*: kernel {statistics.median(ms):.4f} ms, "
          f"effective clock {statistics.median(ghz):.3f} GHz (min {min(ghz):.3f}, max {max(ghz):.3f})")


if __name__ == "__main__":
    main()
