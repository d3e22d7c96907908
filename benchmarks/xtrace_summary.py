#!/usr/bin/env python3
"""Where does a pull's ~590 us go between launch and completion? Reads the
rocprofv3 csv traces of benchmarks/xproc_trace.sh (one dir per rank):

  * per kernel name: dispatches, mean / p50 / p99 duration;
  * for each dispatch, launch API end (hip_api_trace, same correlation id)
    -> kernel start (queueing on the device), and kernel end -> the next
    hipEventQuery/hipEventSynchronize that ends after it on any thread
    (how late the host notices);
  * the per-queue view: how many kernels are busy at once, and which other
    kernels sat on the same queue right before a slow-starting pull.

  python benchmarks/xtrace_summary.py gpurun_out/xtrace/r0 gpurun_out/xtrace/r1 [--prune]
"""
import bisect
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rocprof_summary import short  # noqa: E402


def pct(v, q):
    if not v:
        return 0.0
    v = sorted(v)
    return v[min(len(v) - 1, int(len(v) * q))]


def load(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def summarize(d):
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    at = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)
    if not kt:
        print("# %s: no kernel trace" % d)
        return
    kernels = load(kt[0])
    api = load(at[0]) if at else []
    print("# %s: %d dispatches, %d HIP API records" % (d, len(kernels), len(api)))
    if kernels:
        print("  kernel columns: %s" % ",".join(kernels[0].keys()))
    if api:
        print("  api columns: %s" % ",".join(api[0].keys()))
    launch_end = {}
    queries = []  # end timestamps of event queries / syncs
    fn_count = collections.Counter()
    fn_ns = collections.Counter()
    for r in api:
        fn = r.get("Function") or r.get("Operation") or r.get("Kind", "?")
        try:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        except (KeyError, ValueError):
            continue
        fn_count[fn] += 1
        fn_ns[fn] += e - s
        if "Launch" in fn or "ModuleLaunch" in fn:
            launch_end[r.get("Correlation_Id")] = e
        if fn in ("hipEventQuery", "hipEventSynchronize", "hipStreamSynchronize", "hipStreamQuery"):
            queries.append(e)
    queries.sort()
    print("  HIP API calls (count, mean us):")
    for fn, c in fn_count.most_common(14):
        print("    %-32s %9d %8.2f" % (fn, c, fn_ns[fn] / c / 1e3))
    by_name = collections.defaultdict(list)
    q_delay = collections.defaultdict(list)
    notice = collections.defaultdict(list)
    per_queue = collections.defaultdict(list)
    for r in kernels:
        try:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        except (KeyError, ValueError):
            continue
        n = short(r.get("Kernel_Name", "?"))
        by_name[n].append((e - s) / 1e3)
        per_queue[r.get("Queue_Id", "?")].append((s, e, n))
        le = launch_end.get(r.get("Correlation_Id"))
        if le is not None:
            q_delay[n].append((s - le) / 1e3)
        i = bisect.bisect_left(queries, e)
        if i < len(queries):
            notice[n].append((queries[i] - e) / 1e3)
    print("  per kernel: dispatches, duration mean/p50/p99 us | launch->start p50/p99/mean us | "
          "end->first query after p50/p99 us")
    for n, v in sorted(by_name.items(), key=lambda kv: -len(kv[1])):
        qd, no = q_delay.get(n, []), notice.get(n, [])
        print("    %-34s %7d  %7.1f %7.1f %7.1f | %8.1f %8.1f %8.1f | %7.1f %7.1f" % (
            n, len(v), sum(v) / len(v), pct(v, 0.5), pct(v, 0.99), pct(qd, 0.5), pct(qd, 0.99),
            sum(qd) / len(qd) if qd else 0.0, pct(no, 0.5), pct(no, 0.99)))
    for lst in per_queue.values():
        lst.sort()
    print("  queues: dispatches and kernel names")
    for q, lst in sorted(per_queue.items()):
        names = collections.Counter(x[2] for x in lst)
        print("    queue %-6s %7d  %s" % (q, len(lst), dict(names.most_common(4))))
    # the slowest-starting pulls: what ran on their queue just before
    slow = []
    for r in kernels:
        le = launch_end.get(r.get("Correlation_Id"))
        if le is None:
            continue
        s = int(r["Start_Timestamp"])
        slow.append((s - le, s, r.get("Queue_Id", "?"), short(r.get("Kernel_Name", "?"))))
    slow.sort(reverse=True)
    print("  5 slowest launch->start, with the previous kernel on their queue:")
    for delay, s, q, n in slow[:5]:
        lst = per_queue[q]
        i = bisect.bisect_left(lst, (s,)) - 1
        prev = lst[i] if i >= 0 else None
        print("    %-30s waited %8.1f us; previous on queue %s: %s" % (
            n, delay / 1e3, q, "%s %.1f us long, ended %.1f us before" % (
                prev[2], (prev[1] - prev[0]) / 1e3, (s - prev[1]) / 1e3) if prev else "-"))


def main():
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    for d in args:
        summarize(d)
        if "--prune" in sys.argv:
            for p in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True):
                if "stats" not in os.path.basename(p):
                    os.remove(p)


if __name__ == "__main__":
    main()
