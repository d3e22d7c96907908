"""One rank of a multi-rank RCCL payload plane job on the CPU (stub RCCL,
gloo control plane). Launched by tests/test_rccl_plane_cpu.py through
torch.distributed.run; prints one JSON line per rank.

Every rank runs an echo server and a ParallelChannel fan-out press to ALL
other ranks with host attachments above -rccl_min_bytes, so every ordered
pair carries payloads in both directions at once (the traffic that could
deadlock a FIFO-ordered plane), at 64 KiB and 1 MiB with 50 calls in flight.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="65536,1048576")
    ap.add_argument("--calls", default="200,12")
    ap.add_argument("--concurrency", type=int, default=50)
    ap.add_argument("--window", type=int, default=0, help="-rccl_window_bytes (0: default)")
    ap.add_argument("--out-dir", default="", help="write rank<N>.json here instead of stdout")
    ap.add_argument("--overcrowd-test", action="store_true",
                    help="after the legs, refuse most writes (tiny -socket_max_unwritten_bytes): payloads queued "
                         "for refused requests must be withdrawn or dropped at the receiver, never stashed")
    ap.add_argument("--ring-test", type=float, default=0.0,
                    help="seconds per phase: every rank presses only rank+1 (ring), first with every poster at "
                         "full speed, then with --slow-rank's poster sleeping --slow-delay-us after every group")
    ap.add_argument("--slow-rank", type=int, default=3)
    ap.add_argument("--slow-delay-us", type=int, default=50000)
    ap.add_argument("--abort-test", action="store_true",
                    help="after the legs, rank 1 aborts the plane under traffic; every rank must notice "
                         "within a second and keep serving through the fallback")
    ap.add_argument("--flags", default="", help="extra native flags, name=value[,name=value...]")
    a = ap.parse_args()
    from brpc_amd import native, parallel
    from brpc_amd.models import start_echo_server
    topo = parallel.init_distributed(prefer_gpu=False)
    native.set_flag("fiber_concurrency", "3")
    native.set_flag("rccl_timeout_ms", "30000")
    for kv in [x for x in a.flags.split(",") if x]:
        k, v = kv.split("=", 1)
        native.set_flag(k, v)
    if a.window:
        native.set_flag("rccl_window_bytes", str(a.window))
    up = parallel.init_rccl_plane(topo, library=parallel.stub_library())
    server = start_echo_server("127.0.0.1:0", num_threads=3)
    addrs = parallel.exchange_addresses(server.address, topo)
    # one rank: it presses its own server, so every payload goes to itself
    others = [x for i, x in enumerate(addrs) if i != topo.rank] or [server.address]
    parallel.set_rccl_min_bytes(32768)
    out = {"rank": topo.rank, "world": topo.world_size, "plane_up": bool(up), "legs": []}
    import time
    for size, calls in zip([int(x) for x in a.sizes.split(",")], [int(x) for x in a.calls.split(",")]):
        if calls <= 0:
            continue
        p = native.Press({"server": others[0], "fanout_servers": ",".join(others), "concurrency": a.concurrency,
                          "attachment_size": size, "check_echo": True, "timeout_ms": 60000})
        p.run_requests(min(calls, 20))  # connections and plane hellos up
        p.reset_stats()
        parallel.barrier(topo)
        s0 = parallel.rccl_stats()
        t0 = time.perf_counter()
        p.run_requests(calls)
        dt = time.perf_counter() - t0
        st = p.stats()
        s1 = parallel.rccl_stats()
        out["legs"].append({"size": size, "calls": calls, "success": st["success"], "error": st["error"],
                            "last_error": st["last_error"], "seconds": dt,
                            "sent_payloads": s1["sent_payloads"] - s0["sent_payloads"],
                            "recv_payloads": s1["recv_payloads"] - s0["recv_payloads"],
                            "groups": s1["rounds"] - s0["rounds"],
                            "pair_rounds": s1["pair_rounds"] - s0["pair_rounds"],
                            "withdrawals": s1["withdrawals"] - s0["withdrawals"],
                            "group_us": s1["group_us"] - s0["group_us"],
                            "credit_stalls": s1["credit_stalls"] - s0["credit_stalls"]})
        del p
        parallel.barrier(topo)
    if a.ring_test > 0:
        nxt = addrs[(topo.rank + 1) % topo.world_size]
        out["ring"] = []
        for phase in ("full_speed", "slow_rank"):
            if phase == "slow_rank" and topo.rank == a.slow_rank:
                native.set_flag("rccl_test_poster_delay_us", str(a.slow_delay_us))
            p = native.Press({"server": nxt, "concurrency": a.concurrency, "attachment_size": 65536,
                              "check_echo": True, "timeout_ms": 60000})
            p.run_requests(20)
            p.reset_stats()
            parallel.barrier(topo)
            s0 = parallel.rccl_stats()
            t0 = time.perf_counter()
            p.run_for(a.ring_test)
            dt = time.perf_counter() - t0
            st = p.stats()
            s1 = parallel.rccl_stats()
            out["ring"].append({"phase": phase, "qps": st["success"] / dt, "error": st["error"],
                                "last_error": st["last_error"],
                                "pair_rounds": s1["pair_rounds"] - s0["pair_rounds"],
                                "groups": s1["rounds"] - s0["rounds"],
                                "sent_payloads": s1["sent_payloads"] - s0["sent_payloads"]})
            del p
            parallel.barrier(topo)
            native.set_flag("rccl_test_poster_delay_us", "0")
            parallel.barrier(topo)
    if a.overcrowd_test:
        import time
        p = native.Press({"server": others[0], "fanout_servers": ",".join(others), "concurrency": a.concurrency,
                          "attachment_size": 1 << 20, "timeout_ms": 5000, "max_retry": 0})
        p.run_requests(50)  # connections up and their plane hellos answered
        p.reset_stats()
        s0 = parallel.rccl_stats()
        native.set_flag("socket_max_unwritten_bytes", "1")
        p.run_requests(300)
        st = p.stats()
        del p
        native.set_flag("socket_max_unwritten_bytes", str(64 << 20))
        parallel.barrier(topo)
        # the cancellations ride the next rounds; give them a moment
        deadline = time.perf_counter() + 5
        while parallel.rccl_stats()["stash_payloads"] and time.perf_counter() < deadline:
            time.sleep(0.01)
        s1 = parallel.rccl_stats()
        out["overcrowd_leg"] = {"success": st["success"], "error": st["error"], "last_error": st["last_error"],
                                "withdrawn": s1["withdrawn"] - s0["withdrawn"],
                                "discarded": s1["discarded"] - s0["discarded"],
                                "stash_payloads": s1["stash_payloads"], "stash_bytes": s1["stash_bytes"]}
        parallel.barrier(topo)
        p = native.Press({"server": others[0], "fanout_servers": ",".join(others), "concurrency": a.concurrency,
                          "attachment_size": 65536, "check_echo": True})
        p.run_requests(100)
        st = p.stats()
        out["after_overcrowd_leg"] = {"success": st["success"], "error": st["error"]}
        del p
        parallel.barrier(topo)
    if a.abort_test:
        import threading
        import time
        others_all = ",".join(others)
        p = native.Press({"server": others[0], "fanout_servers": others_all, "concurrency": a.concurrency,
                          "attachment_size": 65536, "check_echo": True, "timeout_ms": 60000})
        th = threading.Thread(target=p.run_for, args=(1.5,))
        parallel.barrier(topo)
        t0 = time.perf_counter()
        th.start()
        time.sleep(0.3)
        if topo.rank == 1:
            native.gpu.rccl_abort_for_test("fault injected by tests/plane_ranks.py")
        t_abort = time.perf_counter()
        while native.gpu.rccl_active() and time.perf_counter() - t_abort < 5:
            time.sleep(0.001)
        out["abort_noticed_ms"] = round(1000 * (time.perf_counter() - t_abort), 1)
        out["plane_active_after_abort"] = bool(native.gpu.rccl_active())
        th.join()
        st = p.stats()
        out["abort_leg"] = {"success": st["success"], "error": st["error"], "elapsed_s": time.perf_counter() - t0}
        del p
        parallel.barrier(topo)
        p = native.Press({"server": others[0], "fanout_servers": others_all, "concurrency": a.concurrency,
                          "attachment_size": 65536, "check_echo": True})
        p.run_requests(100)
        st = p.stats()
        out["after_abort_leg"] = {"success": st["success"], "error": st["error"]}
        del p
        parallel.barrier(topo)
    st = parallel.rccl_stats()
    out["aborts"] = st["aborts"]
    out["sent_payloads"] = st["sent_payloads"]
    out["recv_payloads"] = st["recv_payloads"]
    out["rounds"] = st["rounds"]
    out["stash_expired"] = st["stash_expired"]
    out["recv_timeouts"] = st["recv_timeouts"]
    out["host_memory"] = st["host_memory"]
    parallel.barrier(topo)
    server.stop()
    line = json.dumps(out)
    if a.out_dir:
        with open(os.path.join(a.out_dir, "rank%d.json" % topo.rank), "w") as f:
            f.write(line)
    else:
        sys.stdout.write(line + "\n")
        sys.stdout.flush()
    parallel.barrier(topo)
    parallel.shutdown_rccl_plane()
    parallel.destroy(topo)


if __name__ == "__main__":
    main()
