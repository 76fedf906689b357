"""Effective clock per kernel from one rocprofv3 pass of tools/pmc_clock.sh: for every dispatch,
GRBM_GUI_ACTIVE (summed over the 8 XCDs by rocprofv3) / 8 / (end - start of the kernel trace),
joined on the dispatch id; median and range over the second half of each kernel's dispatches
(after the clocks settled). Prints JSON."""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import kernel_key  # noqa: E402


def rows(root, pattern):
    out = []
    for f in glob.glob(os.path.join(root, "**", pattern), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main(root):
    dur = {}
    for r in rows(root, "*kernel_trace.csv"):
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9, r["Kernel_Name"]
    gui = {}
    for r in rows(root, "*counter_collection.csv"):
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            gui[r["Dispatch_Id"]] = gui.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    per = defaultdict(list)
    for d, (s, name) in sorted(dur.items(), key=lambda kv: int(kv[0])):
        k = kernel_key(name)
        if k and d in gui and s > 0:
            per[k].append((s * 1e6, gui[d] / 8 / s / 1e9))
    out = {}
    for k, v in per.items():
        tail = v[len(v) // 2:]
        ghz = [c for _, c in tail]
        out[k] = {"dispatches": len(v), "median_us": round(statistics.median(u for u, _ in tail), 2),
                  "clock_ghz_median": round(statistics.median(ghz), 3),
                  "clock_ghz_range": [round(min(ghz), 3), round(max(ghz), 3)]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
