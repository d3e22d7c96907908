#!/usr/bin/env python3
"""Where does the time of a paced (100 QPS) 32 B echo go?

Runs the bench's latency sample (one caller, 100 QPS, loopback baidu_std)
with rpcz on, pairs every client span with its server span by trace id and
splits each call into phases:

  issue     call start -> request handed to the socket (client)
  req_wire  request written -> request cut by the server's dispatcher
            (kernel loopback + the server side waking up)
  server    request cut -> response written (server)
  resp_wire response written -> response cut on the client
            (kernel loopback + the client side waking up)
  queue     response cut -> response processing began (client)
  done      processing began -> call ended

  python benchmarks/latency_trace.py --seconds 10
"""
import argparse
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ("issue", "req_wire", "server", "resp_wire", "queue", "done")


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))] if v else 0


def thread_sched():
    """{tid: (name, run_ns, runqueue_wait_ns, involuntary switches, cpu)} of this process."""
    out = {}
    base = "/proc/self/task"
    for tid in os.listdir(base):
        try:
            with open("%s/%s/schedstat" % (base, tid)) as f:
                run, wait, _ = (int(x) for x in f.read().split())
            with open("%s/%s/comm" % (base, tid)) as f:
                name = f.read().strip()
            nonvol = 0
            with open("%s/%s/status" % (base, tid)) as f:
                for line in f:
                    if line.startswith("nonvoluntary_ctxt_switches"):
                        nonvol = int(line.split()[1])
            with open("%s/%s/stat" % (base, tid)) as f:
                cpu = int(f.read().rsplit(")", 1)[1].split()[36])
            out[tid] = (name, run, wait, nonvol, cpu)
        except (OSError, ValueError, IndexError):
            pass
    return out


def cpu_irq_ticks():
    """{cpu: (irq + softirq ticks, total ticks)} from /proc/stat."""
    out = {}
    try:
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("cpu") and line[3].isdigit():
                    v = line.split()
                    t = list(map(int, v[1:]))
                    out[int(v[0][3:])] = (t[5] + t[6], sum(t))
    except OSError:
        pass
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--qps", type=float, default=100.0)
    ap.add_argument("--workers", type=int, default=12)
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--attachment", type=int, default=0, help="attachment bytes per call")
    ap.add_argument("--device-attachment", action="store_true", help="attachment in HBM (lent over xGMI)")
    ap.add_argument("--gpu-process", action="store_true", help="the server runs the GPU handler over the attachment")
    ap.add_argument("--concurrency", type=int, default=1)
    ap.add_argument("--dump", type=int, default=0, help="print the full spans of this many slowest calls")
    a = ap.parse_args()
    import torch
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    native.set_flag("fiber_concurrency", str(a.workers))
    if "L3_DOMAIN" in os.environ:
        native.set_flag("cpu_l3_domain", os.environ["L3_DOMAIN"])
    elif torch.cuda.is_available():
        from brpc_amd.parallel.placement import choose_l3_domain
        l3, _ = choose_l3_domain(0, 1, 0, torch.cuda.device_count())
        if l3 >= 0:
            native.set_flag("cpu_l3_domain", str(l3))
    native.set_flag("event_dispatcher_spin_us", os.environ.get("SPIN_US", "200"))
    if "NAP_US" in os.environ:
        native.set_flag("event_dispatcher_nap_us", os.environ["NAP_US"])
    if "WORKER_NAP_US" in os.environ:
        native.set_flag("fiber_worker_nap_us", os.environ["WORKER_NAP_US"])
    native.set_flag("rpcz_save_to_disk", "false")
    native.set_flag("rpcz_max_spans", "100000")
    native.set_flag("rpcz_max_spans_per_second", "100000")
    dev = 0 if (a.device_attachment or a.gpu_process) else -1
    s = start_echo_server("127.0.0.1:0", num_threads=a.workers, gpu_device=dev)
    o = {"server": s.address, "qps": a.qps, "concurrency": a.concurrency, "request_size": 32,
         "connection_type": "single"}
    if a.attachment:
        o.update({"attachment_size": a.attachment, "gpu_device": dev, "device_attachment": a.device_attachment,
                  "gpu_process": a.gpu_process})
    p = native.Press(o)
    p.run_for(0.5)
    if not os.environ.get("NO_RPCZ"):
        native.set_flag("enable_rpcz", "true")
    p.reset_stats()
    t0, q0 = thread_sched(), cpu_irq_ticks()
    p.run_for(a.seconds)
    t1, q1 = thread_sched(), cpu_irq_ticks()
    native.set_flag("enable_rpcz", "false")
    st = p.stats()
    if dev >= 0:
        x = native.gpu.xgmi_stats()
        print("hbm pool:", native.gpu.hbm_pool_stats(0))
        print("xgmi:", {k: x[k] for k in ("sent_payloads", "recv_payloads", "copied_into_arena", "ring_full_fallbacks",
                                          "copy_launches", "copy_segments", "copy_submits", "copy_queue_us",
                                          "copy_api_us", "copy_gpu_us", "copy_wake_us")})
    spans = native.rpcz_recent(1000000)
    client, server, raw = {}, {}, {}
    for d in spans:
        head = d.split("\n", 1)[0]
        m = re.search(r"trace=([0-9a-f]+)", head)
        if not m:
            continue
        kv = {k: int(v) for k, v in re.findall(r" (\w+)=\+?(-?\d+)(?:us)?(?= |$)", head)}
        (client if head.startswith("C ") else server)[m.group(1)] = kv
        raw.setdefault(m.group(1), []).append(d)
    rows = []
    for t, c in client.items():
        sv = server.get(t)
        if not sv or "sent" not in c or "cut" not in c:
            continue
        start = c["start"]
        srv_recv, srv_sent = sv["received"], sv["received"] + sv["sent"]
        ph = {
            "issue": c["sent"],
            "req_wire": srv_recv - (start + c["sent"]),
            "server": srv_sent - srv_recv,
            "resp_wire": start + c["cut"] - srv_sent,
            "queue": c["parse"] - c["cut"],
            "done": c["latency"] - c["parse"],
        }
        rows.append((c["latency"], ph, t))
    print("press: qps=%.0f p50=%s p99=%s p999=%s; traced calls=%d" % (st["qps"], st["p50_us"], st["p99_us"],
                                                                     st["p999_us"], len(rows)))
    lat = [r[0] for r in rows]
    print("traced latency: p50=%d p90=%d p99=%d max=%d us" % (pct(lat, .5), pct(lat, .9), pct(lat, .99),
                                                              max(lat) if lat else 0))
    print("%-10s %6s %6s %6s %6s" % ("phase", "p50", "p90", "p99", "max"))
    for k in PHASES:
        v = [r[1][k] for r in rows]
        print("%-10s %6d %6d %6d %6d" % (k, pct(v, .5), pct(v, .9), pct(v, .99), max(v) if v else 0))
    # were our threads runnable but not running (preempted by other tasks),
    # and how much of their CPUs went to interrupts?
    rows_t = []
    for tid, (name, run, wait, nonvol, cpu) in t1.items():
        b = t0.get(tid)
        if b:
            rows_t.append((wait - b[2], run - b[1], nonvol - b[3], name, cpu))
    rows_t.sort(reverse=True)
    print("sched: runqueue wait %.2f ms, run %.2f ms, involuntary switches %d over %d threads; worst: %s" % (
        sum(r[0] for r in rows_t) / 1e6, sum(r[1] for r in rows_t) / 1e6, sum(r[2] for r in rows_t), len(rows_t),
        ", ".join("%s@%d wait=%.2fms nonvol=%d" % (r[3], r[4], r[0] / 1e6, r[2]) for r in rows_t[:4])))
    cpus = sorted(os.sched_getaffinity(0))
    irq = [(q1[c][0] - q0[c][0]) / max(1, q1[c][1] - q0[c][1]) for c in cpus if c in q0 and c in q1]
    print("irq+softirq share of our CPUs: mean %.2f%% max %.2f%%" % (100 * sum(irq) / max(1, len(irq)),
                                                                   100 * max(irq + [0])))
    print("slowest calls:")
    slowest = sorted(rows, key=lambda r: -r[0])
    for latency, ph, _ in slowest[:a.top]:
        print("  %5d us: " % latency + " ".join("%s=%d" % (k, ph[k]) for k in PHASES))
    for _, _, t in slowest[:a.dump]:
        print("--- trace %s" % t)
        for d in raw.get(t, []):
            print(d)
    s.stop()


if __name__ == "__main__":
    main()
