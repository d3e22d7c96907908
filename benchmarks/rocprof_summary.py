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
    """Kernel name without return type, namespaces or argument list:
    'void mrpc::gpu::(anonymous namespace)::copy_crc32c_kernel(SegBatch, ...)'
    -> 'copy_crc32c_kernel'. Parentheses and '<>' nest, so the argument list
    is the first '(' at depth 0 after the name (not '(anonymous namespace)')."""
    n = name.replace("(anonymous namespace)::", "").strip()
    if n.startswith("void "):
        n = n[5:]
    depth, cut = 0, len(n)
    for i, c in enumerate(n):
        if c == "<":
            depth += 1
        elif c == ">":
            depth -= 1
        elif c == "(" and depth == 0:
            cut = i
            break
    n = n[:cut]
    # last component at template depth 0
    depth, start = 0, 0
    for i, c in enumerate(n):
        if c == "<":
            depth += 1
        elif c == ">":
            depth -= 1
        elif c == ":" and depth == 0 and i + 1 < len(n) and n[i + 1] == ":":
            start = i + 2
    return (n[start:] or name)[:56]


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
        # overlap: the union of kernel busy intervals against the sum of
        # their durations (1.0 = kernels never overlap), and per-queue stats
        for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            iv, queues = [], collections.Counter()
            with open(p) as f:
                for r in csv.DictReader(f):
                    try:
                        iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
                    except (KeyError, ValueError):
                        continue
                    queues[r.get("Queue_Id", "?")] += 1
            if not iv:
                continue
            iv.sort()
            busy, cur_s, cur_e = 0, iv[0][0], iv[0][1]
            for s0, e0 in iv[1:]:
                if s0 > cur_e:
                    busy += cur_e - cur_s
                    cur_s, cur_e = s0, e0
                else:
                    cur_e = max(cur_e, e0)
            busy += cur_e - cur_s
            total = sum(e0 - s0 for s0, e0 in iv)
            span = iv[-1][1] - iv[0][0]
            print("## overlap (%s): %d dispatches over %.1f ms, GPU busy %.1f ms (%.0f%% of the span), "
                  "sum of durations %.1f ms, mean concurrency when busy %.2f, queues %s" % (
                      os.path.basename(p), len(iv), span / 1e6, busy / 1e6, 100.0 * busy / max(1, span),
                      total / 1e6, total / max(1, busy), dict(queues)))
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
