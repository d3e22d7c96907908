#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (run_results.db) into a per-kernel
table: calls, total/avg/min/max duration. Usage: rocprof_summary.py DB [OUT]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else None)
    q = ("select %s as k, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
         "from kernels group by k order by sum(end-start) desc" % name_col)
    rows = list(c.execute(q))
    total = sum(r[2] for r in rows) or 1
    lines = ["%-90s %8s %12s %10s %10s %10s %6s" % ("kernel", "calls", "total_us", "avg_us", "min_us", "max_us", "pct")]
    for k, n, tot, avg, mn, mx in rows:
        k = (k or "?")
        if len(k) > 88:
            k = k[:85] + "..."
        lines.append("%-90s %8d %12.1f %10.2f %10.2f %10.2f %5.1f%%" % (k, n, tot / 1e3, avg / 1e3, mn / 1e3, mx / 1e3,
                                                                        100.0 * tot / total))
    out = "\n".join(lines) + "\n"
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(out)
    print(out)


if __name__ == "__main__":
    main()
