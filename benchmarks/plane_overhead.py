#!/usr/bin/env python3
"""CPU overhead curve of the RCCL payload plane (csrc/gpu/rccl_plane.h) on the
stub RCCL (bounded shm FIFOs, host memory): 2/4/8 ranks fan 64 KiB
attachments out to every other rank (both directions of every pair busy),
then an 8-rank ring with and without one slow poster.

This is a CPU overhead curve of the plane's control path (pair rounds over
shm, one group per rank in flight), not a scaling claim: the stub moves
bytes with memcpy through 64 KiB FIFOs on a shared host.

  python benchmarks/plane_overhead.py > profiles/r4_rccl_plane_overhead.txt
"""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


FLAGS = []


def run(nranks, port, *extra):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
                            str(nranks), "--master-addr", "127.0.0.1", "--master-port", str(port),
                            os.path.join(ROOT, "tests", "plane_ranks.py"), "--out-dir", d] + FLAGS + list(extra),
                           capture_output=True, text=True, timeout=900, cwd="/tmp", env=env)
        if r.returncode != 0:
            raise SystemExit(r.stderr[-3000:])
        return [json.load(open(os.path.join(d, "rank%d.json" % k))) for k in range(nranks)]


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--repeat", type=int, default=1)
    ap.add_argument("--no-ring", action="store_true")
    ap.add_argument("--flags", default="", help="native flags for every rank, name=value[,...]")
    a = ap.parse_args()
    if a.flags:
        FLAGS.extend(["--flags", a.flags])
        print("# flags: %s" % a.flags)
    print("# RCCL plane overhead on the stub library (fan-out: every rank -> every other rank, 50 in flight)")
    print("%-6s %-8s %-10s %-10s %-12s %-12s %-14s %-14s %-10s" % (
        "ranks", "size", "calls/s", "payloads", "groups/s", "pair_rnds/s", "payloads/grp", "us/payload",
        "withdraw"))
    ports = {2: 29700, 4: 29710, 8: 29720}
    for n in [int(x) for x in a.ranks.split(",")] * a.repeat:
        outs = run(n, ports.get(n, 29740 + n), "--sizes", "65536,1048576", "--calls", "400,40")
        for k in range(2):
            legs = [o["legs"][k] for o in outs]
            secs = max(l["seconds"] for l in legs)
            calls = sum(l["success"] for l in legs)
            pay = sum(l["sent_payloads"] for l in legs)
            groups = sum(l["groups"] for l in legs)
            prs = sum(l["pair_rounds"] for l in legs) / 2.0  # each pair round is counted by both sides
            wd = sum(l["withdrawals"] for l in legs)
            print("%-6d %-8d %-10.0f %-10d %-12.0f %-12.0f %-14.2f %-14.1f %-10d" % (
                n, legs[0]["size"], calls / secs, pay, groups / secs / n, prs / secs, pay / max(1, groups),
                1e6 * secs * n / max(1, pay), wd))
    if a.no_ring:
        return
    print()
    print("# 8-rank ring (rank r -> r+1, 64 KiB), then rank 3's poster sleeping 50 ms after every group")
    outs = run(8, 29730, "--calls", "0,0", "--ring-test", "2", "--slow-rank", "3", "--slow-delay-us", "50000")
    print("%-6s %-14s %-14s %-8s %s" % ("rank", "qps_full", "qps_slow_rank3", "ratio", "pair"))
    for o in outs:
        f, s = o["ring"]
        r = o["rank"]
        print("%-6d %-14.0f %-14.0f %-8.2f %d->%d%s" % (r, f["qps"], s["qps"], s["qps"] / max(1.0, f["qps"]), r,
                                                       (r + 1) % 8, "  (includes rank 3)" if r in (2, 3) else ""))


if __name__ == "__main__":
    main()
