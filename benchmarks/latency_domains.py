#!/usr/bin/env python3
"""100-QPS 32 B echo latency per L3 domain of the host.

The bench confines a rank to one L3 domain; which one decides the tail of
its paced latency sample (other jobs' threads on those CPUs preempt ours,
and idle domains sleep deeper). For every domain this runs the tracer in a
child process confined there and prints the domain's NUMA node, how busy
the rest of the host kept it just before, and the p50/p99/p999.

  python benchmarks/latency_domains.py --seconds 4
"""
import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--domains", default="", help="comma list (default: all)")
    ap.add_argument("--repeat", type=int, default=1)
    ap.add_argument("--env", default="", help="extra env for the tracer, e.g. WORKER_NAP_US=50,NO_RPCZ=1")
    a = ap.parse_args()
    from brpc_amd.parallel.placement import cpu_busy, l3_domains, numa_nodes
    doms = l3_domains()
    nodes = numa_nodes()
    pick = [int(x) for x in a.domains.split(",")] if a.domains else list(range(len(doms)))
    print("domain first_cpu node busy_pct qps p50 p99 p999 traced_p99 issue_p99 req_wire_p99 resp_wire_p99 "
          "rq_wait_ms nonvol irq_pct", flush=True)
    for _ in range(a.repeat):
        for i in pick:
            cpus = doms[i][1]
            node = next((n for n, cs in nodes.items() if set(cpus) <= cs), -1)
            busy = cpu_busy(0.2)
            b = 100.0 * sum(busy.get(c, 0.0) for c in cpus) / len(cpus) if busy else -1
            env = dict(os.environ, L3_DOMAIN=str(i))
            if a.env:
                env.update(dict(kv.split("=", 1) for kv in a.env.split(",")))
            r = subprocess.run(["timeout", "-k", "5", str(int(a.seconds + 60)), sys.executable,
                                os.path.join(ROOT, "benchmarks", "latency_trace.py"), "--seconds", str(a.seconds),
                                "--top", "0"], env=env, capture_output=True, text=True)
            out = r.stdout
            m = re.search(r"press: qps=(\d+) p50=(\d+) p99=(\d+) p999=(\d+)", out)
            t = re.search(r"traced latency: p50=\d+ p90=\d+ p99=(\d+)", out)
            ph = {k: re.search(r"^%s\s+\d+\s+\d+\s+(\d+)" % k, out, re.M) for k in ("issue", "req_wire", "resp_wire")}
            sch = re.search(r"sched: runqueue wait ([\d.]+) ms, run [\d.]+ ms, involuntary switches (\d+)", out)
            iq = re.search(r"irq\+softirq share of our CPUs: mean ([\d.]+)%", out)
            extra = "%s %s %s" % (sch.group(1) if sch else "-", sch.group(2) if sch else "-", iq.group(1) if iq else "-")
            if r.returncode != 0 or not m:
                print("%d %d %d rc=%d %s" % (i, doms[i][0], node, r.returncode, (r.stderr or out)[-300:]), flush=True)
                continue
            print("%d %d %d %.1f %s %s %s %s %s %s %s %s %s" % (
                i, doms[i][0], node, b, m.group(1), m.group(2), m.group(3), m.group(4), t.group(1) if t else "-",
                *(ph[k].group(1) if ph[k] else "-" for k in ("issue", "req_wire", "resp_wire")), extra), flush=True)


if __name__ == "__main__":
    main()
