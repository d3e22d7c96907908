#!/usr/bin/env python3
"""CPU profile of one echo leg (where do the host cycles of an RPC go?).

Runs a closed-loop press in a Python thread while the in-process sampling
profiler (csrc/builtin/cpu_profiler.cc, SIGPROF + backtrace) records every
thread, then prints the hottest frames by self and inclusive samples.

  python benchmarks/profile_leg.py --leg gpu_handler --seconds 3
"""
import argparse
import collections
import os
import sys
import resource
import threading
import time


def cgroup_cpu_stat():
    """cgroup v2 cpu.stat counters (nr_throttled, throttled_usec, ...)."""
    out = {}
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for line in f:
                k, v = line.split()
                out[k] = int(v)
    except (OSError, ValueError):
        pass
    return out

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--leg", default="gpu_handler",
                    choices=["gpu_handler", "host_64k", "dev_64k", "echo_32b", "rccl_64k", "lat_100qps", "grpc_cpu",
                             "grpc_gpu", "baidu_cpu", "baidu_gpu", "ids_baidu_cpu", "ids_baidu_gpu", "ids_json_cpu", "ids_json_gpu", "dev_snappy", "grpc_dev_snappy", "grpc_dev_64k", "dev_64k_verify",
                             "dev_1m_verify"])
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--body", default="text", help="echo body kind of the codec legs: text, random, const")
    ap.add_argument("--concurrency", type=int, default=50)
    ap.add_argument("--workers", type=int, default=12)
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--folded-out", default="")
    ap.add_argument("--no-profile", action="store_true", help="just run the leg (no SIGPROF sampling)")
    ap.add_argument("--flags", default="", help="comma-separated name=value runtime flags to set first")
    a = ap.parse_args()
    import torch
    from brpc_amd import native, parallel
    from brpc_amd.models import start_echo_server
    cuda = torch.cuda.is_available()
    native.set_flag("fiber_concurrency", str(a.workers))
    for kv in filter(None, a.flags.split(",")):
        k, _, v = kv.partition("=")
        native.set_flag(k, v)
    dev = 0 if cuda else -1
    if cuda:
        from brpc_amd.parallel.placement import choose_l3_domain
        l3, _ = choose_l3_domain(0, 1, 0, torch.cuda.device_count())
        if l3 >= 0:
            native.set_flag("cpu_l3_domain", str(l3))
    native.set_flag("event_dispatcher_spin_us", os.environ.get("SPIN_US", "200"))
    if os.environ.get("RESIDENT"):
        native.set_flag("copy_engine_resident", "true")
        if os.environ.get("RESIDENT_GROUPS"):
            native.set_flag("copy_engine_resident_groups", os.environ["RESIDENT_GROUPS"])
    if "NAP_US" in os.environ:
        native.set_flag("event_dispatcher_nap_us", os.environ["NAP_US"])
    native.set_flag("gpu_poller_idle_spin_us", os.environ.get("POLL_SPIN_US", os.environ.get("SPIN_US", "200")))
    topo = parallel.Topology(rank=0, world_size=1, local_rank=0, local_world_size=1, device=dev)
    if a.leg == "rccl_64k":
        parallel.init_rccl_plane(topo, min_bytes=32768)
    s = start_echo_server("127.0.0.1:0", num_threads=a.workers, gpu_device=dev)
    o = {"server": s.address, "concurrency": a.concurrency, "request_size": 16, "gpu_device": dev}
    if a.leg in ("gpu_handler", "host_64k", "dev_64k", "rccl_64k"):
        o["attachment_size"] = 65520
    if a.leg == "gpu_handler":
        o["gpu_process"] = True
    if a.leg in ("dev_64k", "rccl_64k"):
        o["device_attachment"] = True
    if a.leg == "grpc_dev_64k":
        o.update({"attachment_size": 65536, "device_attachment": True, "protocol": "h2:grpc"})
    if a.leg in ("dev_snappy", "grpc_dev_snappy"):
        # the bench's [grpc_]device_snappy_64KB_<body> leg: an HBM protobuf body
        # encoded/decoded/indexed on the device both ways
        o.update({"attachment_size": 65536, "device_attachment": True, "attachment_body": a.body,
                  "attachment_pb": True, "device_scan": True, "device_compress": 1})
        if a.leg == "grpc_dev_snappy":
            o["protocol"] = "h2:grpc"
    if a.leg == "dev_64k_verify":
        o.update({"attachment_size": 65536, "device_attachment": True, "verify_device_payload": True})
    if a.leg == "dev_1m_verify":
        # 1 MiB HBM attachments, CRC32C-verified on the device (fused into the pull)
        o.update({"attachment_size": 1 << 20, "device_attachment": True, "verify_device_payload": True})
    if a.leg == "echo_32b":
        o["request_size"] = 32
    if a.leg == "lat_100qps":
        o.update({"qps": 100.0, "concurrency": 1, "request_size": 32})
    if a.leg in ("grpc_cpu", "grpc_gpu"):
        # the bench's gRPC + snappy leg: 64 KiB protobuf body, snappy both ways
        o.update({"request_size": 65536, "protocol": "h2:grpc", "request_compress_type": 1})
        if a.leg == "grpc_gpu":
            native.gpu.enable_snappy(dev, 16384)
    if a.leg.startswith("baidu_"):
        # the bench's baidu_std + snappy 64 KiB leg
        o.update({"request_size": 65536, "protocol": "baidu_std", "request_compress_type": 1})
        if a.leg == "baidu_gpu":
            native.gpu.enable_snappy(dev, 16384)
    if a.leg.startswith("ids_"):
        # the bench's 16k packed-ids legs: device pack/unpack with snappy
        # (baidu_std) or device pb2json/json2pb number arrays (http + json)
        o.update({"request_size": 16, "packed_ids": 16384})
        if a.leg.startswith("ids_baidu"):
            o.update({"protocol": "baidu_std", "request_compress_type": 1})
            if a.leg.endswith("gpu"):
                native.gpu.enable_snappy(dev, 16384)
        else:
            o.update({"protocol": "http", "connection_type": "pooled"})
            if a.leg.endswith("gpu"):
                native.gpu.enable_json_index(dev, 16384)
    o["body"] = a.body
    p = native.Press(o)
    p.run_for(0.5)
    p.reset_stats()
    th = threading.Thread(target=p.run_for, args=(a.seconds + 0.4,))
    c0 = cgroup_cpu_stat()
    x0 = native.gpu.xgmi_stats()
    t0 = time.perf_counter()
    r0 = resource.getrusage(resource.RUSAGE_SELF)
    th.start()
    if a.no_profile:
        time.sleep(a.seconds)
        folded, n = "", 0
    else:
        folded, n = native.profile_cpu(a.seconds, 999)
    th.join()
    r1 = resource.getrusage(resource.RUSAGE_SELF)
    wall = time.perf_counter() - t0
    c1 = cgroup_cpu_stat()
    st = p.stats()
    cpu = (r1.ru_utime - r0.ru_utime + r1.ru_stime - r0.ru_stime) / wall
    thr = {k: c1.get(k, 0) - c0.get(k, 0) for k in ("nr_throttled", "throttled_usec", "nr_periods")}
    print("leg=%s qps=%.0f p50=%s p99=%s errors=%d samples=%d cpus_used=%.2f cgroup=%s" % (
        a.leg, st["qps"], st["p50_us"], st["p99_us"], st["error"], n, cpu, thr))
    if st["error"]:
        print("last_error:", st.get("last_error"), "codes:", st.get("error_codes"))
    x1 = native.gpu.xgmi_stats()
    if a.leg.endswith("dev_snappy"):
        print("device codec:", native.gpu.device_codec_stats(), "codec batch:", native.gpu.codec_batch_stats())
    if os.environ.get("RESIDENT"):
        print("resident:", native.gpu.resident_stats())
    subs = x1["copy_submits"] - x0["copy_submits"]
    if subs:
        print("copy engine per submission: queue %.1f us, launch API %.1f us, GPU+poll %.1f us, wake %.1f us; "
              "%.2f submissions/launch" % tuple(
                  [(x1[k] - x0[k]) / subs for k in ("copy_queue_us", "copy_api_us", "copy_gpu_us", "copy_wake_us")] +
                  [subs / max(1, x1["copy_launches"] - x0["copy_launches"])]))
    if a.folded_out:
        with open(a.folded_out, "w") as f:
            f.write(folded)
    self_c, incl_c = collections.Counter(), collections.Counter()
    total = 0
    for line in folded.splitlines():
        stack, _, cnt = line.rpartition(" ")
        try:
            c = int(cnt)
        except ValueError:
            continue
        frames = stack.split(";")
        total += c
        self_c[frames[-1]] += c
        for f in set(frames):
            incl_c[f] += c
    print("--- self (of %d samples)" % total)
    for f, c in self_c.most_common(a.top):
        print("%6.2f%%  %s" % (100.0 * c / max(1, total), f[:160]))
    print("--- inclusive")
    for f, c in incl_c.most_common(a.top):
        print("%6.2f%%  %s" % (100.0 * c / max(1, total), f[:160]))
    s.stop()


if __name__ == "__main__":
    main()
