#!/usr/bin/env python3
"""Summarise a rocprofv3 output directory (csv format) into a small text
table — per kernel (and grid size): dispatches, mean duration, and for PMC
runs the mean counter values with the achieved bandwidth of FETCH_SIZE /
WRITE_SIZE (KiB per dispatch) against 8 TB/s HBM3E. With --prune the large
per-dispatch CSVs are deleted afterwards (gpurun copies back <= 64 MiB).

  python benchmarks/rocprof_summary.py gpurun_out/b/pmc_fetch_handler --prune > summary.txt
"""
import argparse
import collections
import csv
import glob
import os
import sys

HBM_GBPS = 8000.0


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    n = n.split("(")[0].strip()
    return n.split("::")[-1][:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--prune", action="store_true")
    a = ap.parse_args()
    for d in a.dirs:
        print("# %s" % d)
        stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
        for p in stats:
            with open(p) as f:
                rows = list(csv.DictReader(f))
            print("## kernel stats (%s)" % os.path.basename(p))
            for r in rows[:25]:
                print("%-48s calls=%-8s total_ms=%-10.3f avg_us=%-9.2f pct=%s" % (
                    short(r.get("Name", "")), r.get("Calls"), float(r.get("TotalDurationNs", 0)) / 1e6,
                    float(r.get("AverageNs", 0)) / 1e3, r.get("Percentage")))
        cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        for p in cc:
            groups = collections.defaultdict(lambda: {"n": set(), "sum": collections.Counter(), "dur": 0.0})
            durs = {}
            with open(p) as f:
                for r in csv.DictReader(f):
                    key = (short(r.get("Kernel_Name", "")), r.get("Grid_Size", ""))
                    g = groups[key]
                    did = r.get("Dispatch_Id") or r.get("Correlation_Id")
                    g["n"].add(did)
                    g["sum"][r.get("Counter_Name", "")] += float(r.get("Counter_Value", 0) or 0)
                    if r.get("Start_Timestamp") and r.get("End_Timestamp") and did not in durs:
                        durs[did] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                        g["dur"] += durs[did]
            print("## counters (%s)" % os.path.basename(p))
            for (k, grid), g in sorted(groups.items(), key=lambda kv: -len(kv[1]["n"])):
                n = max(1, len(g["n"]))
                parts = ["%s=%.1f" % (c, v / n) for c, v in sorted(g["sum"].items())]
                line = "%-48s grid=%-9s dispatches=%-7d" % (k, grid, n)
                if g["dur"] > 0:
                    dur = g["dur"] / n
                    kib = sum(v for c, v in g["sum"].items() if c in ("FETCH_SIZE", "WRITE_SIZE")) / n
                    gbps = kib * 1024 / (dur * 1e-6) / 1e9 if dur > 0 else 0
                    line += " dur_us=%-8.2f %s GB/s=%.1f (%.1f%% of 8 TB/s)" % (dur, " ".join(parts), gbps,
                                                                              100 * gbps / HBM_GBPS)
                else:
                    line += " " + " ".join(parts)
                print(line)
        if a.prune:
            for p in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True):
                if not p.endswith("kernel_stats.csv") and not p.endswith("agent_info.csv"):
                    os.remove(p)
            for p in glob.glob(os.path.join(d, "**", "*.db"), recursive=True) + \
                    glob.glob(os.path.join(d, "**", "*.json"), recursive=True):
                os.remove(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())
