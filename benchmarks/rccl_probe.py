#!/usr/bin/env python3
"""One rank, the RCCL payload plane only: device-attachment echo of the
given sizes / queue depths for a fixed time each, with the plane's counters
and the HBM pool after every point (diagnoses plane stalls and memory).

  python benchmarks/rccl_probe.py --points 16777216:16,16777216:1,8388608:16
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", default="16777216:16")
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--timeout-ms", type=int, default=5000)
    a = ap.parse_args()
    import torch  # noqa: F401
    from brpc_amd import native, parallel
    from brpc_amd.models import start_echo_server
    topo = parallel.Topology(rank=0, world_size=1, local_rank=0, local_world_size=1, device=0)
    assert parallel.init_rccl_plane(topo, min_bytes=32768)
    srv = start_echo_server("127.0.0.1:0", gpu_device=0)
    for pt in a.points.split(","):
        size, qd = (int(x) for x in pt.split(":"))
        p = native.Press({"server": srv.address, "concurrency": qd, "attachment_size": size, "request_size": 16,
                          "device_attachment": True, "gpu_device": 0, "timeout_ms": a.timeout_ms, "max_retry": 0})
        r0 = parallel.rccl_stats()
        x0 = native.gpu.xgmi_stats()
        t0 = time.perf_counter()
        p.run_for(a.seconds)
        dt = time.perf_counter() - t0
        st = p.stats()
        r1 = parallel.rccl_stats()
        x1 = native.gpu.xgmi_stats()
        xd = {k: x1[k] - x0[k] for k in ("sent_payloads", "recv_payloads", "staged_payloads", "ring_full_fallbacks")}
        d = {k: r1[k] - r0[k] for k in r1 if isinstance(r1[k], int) and r1[k] != r0[k]}
        hb = native.gpu.hbm_pool_stats(0)
        print("size=%d qd=%d ok=%d err=%d qps=%.0f p99=%s last=%s | rccl %s | xgmi %s | hbm live=%d fallback=%d" % (
            size, qd, st["success"], st["error"], st["success"] / dt, st["p99_us"], st["last_error"][:100], d, xd,
            hb["live_blocks"], hb["fallback_allocs"]), flush=True)
        del p
    srv.stop()
    parallel.shutdown_rccl_plane()


if __name__ == "__main__":
    main()
