#!/usr/bin/env python3
"""Diagnose the tail of the 100-QPS latency sample: runs the bench's
rpc_press -qps=100 workload (same runtime settings as bench.py) and reports
when the slow calls happen (phase within each second, gaps between them)."""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--slow-us", type=int, default=80)
    ap.add_argument("--l3", type=int, default=1)
    ap.add_argument("--poll-us", type=int, default=1000000)
    ap.add_argument("--workers", type=int, default=12)
    ap.add_argument("--flags", default="")
    a = ap.parse_args()
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    native.set_flag("fiber_concurrency", str(a.workers))
    if a.l3 >= 0:
        native.set_flag("cpu_l3_domain", str(a.l3))
    native.set_flag("event_dispatcher_spin_us", str(a.poll_us))
    native.set_flag("press_slow_trace_us", str(a.slow_us))
    for item in a.flags.split():
        k, _, v = item.lstrip("-").partition("=")
        native.set_flag(k, v or "true")
    s = start_echo_server("127.0.0.1:0", num_threads=a.workers)
    p = native.Press({"server": s.address, "qps": 100.0, "concurrency": 1, "request_size": 32,
                      "connection_type": "single"})
    native.press_slow_calls()
    t_start = native.monotonic_us()
    p.run_for(a.seconds)
    st = p.stats()
    slow = native.press_slow_calls()
    print("calls=%d p50=%s p99=%s avg=%s slow(>=%dus)=%d" % (st["success"], st["p50_us"], st["p99_us"],
                                                            st["avg_us"], a.slow_us, len(slow)))
    phases = collections.Counter()
    prev = None
    gaps = []
    for t0, lat in slow:
        phases[((t0 - t_start) % 1000000) // 100000] += 1
        if prev is not None:
            gaps.append((t0 - prev) / 1000.0)
        prev = t0
    print("slow latencies (us):", sorted(l for _, l in slow)[-20:])
    print("phase within second (100ms bins):", dict(sorted(phases.items())))
    print("gaps between slow calls (ms):", [round(g, 1) for g in gaps[:40]])
    s.stop()


if __name__ == "__main__":
    main()
