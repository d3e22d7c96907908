#!/usr/bin/env python3
"""Snappy kernels at RPC batch shapes: per-launch kernel time of the piece
decoder and the block encoder on a batch of 64 KiB bodies cut into 4 KiB
pieces (the gRPC / baidu_std GPU-codec legs), with the compressed stream and
the output in HBM or in pinned host memory (the RPC path's direct mode).

Prints one JSON line per (kernel, body, input placement, output placement).
Bodies: 'text' (service-log records like press.cc's text body, ~3:1) and
'random' (incompressible).

  python benchmarks/snappy_rpc_shapes.py [--bodies 7] [--iters 50]
"""
import argparse
import json
import os
import random
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def text_body(size, seed):
    rnd = random.Random(seed)
    levels = ["INFO", "INFO", "INFO", "WARN", "DEBUG", "ERROR"]
    paths = ["/api/v1/items", "/api/v1/users", "/api/v2/search", "/healthz", "/api/v1/orders", "/static/app.js",
             "/api/v2/cart", "/login"]
    users = ["alice", "bob", "carol", "dave", "erin", "frank", "grace", "heidi", "ivan", "judy"]
    agents = ["curl/8.5.0", "Mozilla/5.0 (X11; Linux x86_64)", "python-requests/2.31", "grpc-go/1.62.0"]
    out, ts = [], 1792242500000000
    n = 0
    while n < size:
        ts += rnd.randrange(5000)
        r = rnd.getrandbits(64)
        i = rnd.getrandbits(64)
        line = ('{"ts":%d,"level":"%s","rank":%d,"req":"%016x","user":"%s","path":"%s/%d","status":%d,'
                '"latency_us":%d,"bytes":%d,"agent":"%s"}\n' % (
                    ts, levels[r % 6], (r >> 8) % 8, i, users[(r >> 12) % 10], paths[(r >> 16) % 8],
                    (r >> 20) % 100000, 200 if (r >> 40) % 10 else 404, (r >> 24) % 20000, (i >> 7) % 1000000,
                    agents[(r >> 44) % 4]))
        out.append(line)
        n += len(line)
    return "".join(out).encode()[:size]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bodies", type=int, default=7, help="64 KiB bodies per launch (RPC batch)")
    ap.add_argument("--block", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--kinds", default="text,random,const")
    ap.add_argument("--flag", action="append", default=[], help="NAME=VALUE runtime flag (repeatable)")
    ap.add_argument("--compress-only", action="store_true")
    ap.add_argument("--places", default="hbm", help="input/output placements to run: hbm or hbm,pinned")
    a = ap.parse_args()
    from brpc_amd import native
    for f in a.flag:
        k, v = f.split("=", 1)
        native.set_flag(k, v)
    from brpc_amd.ops._common import stream_handle
    dev = torch.device("cuda", 0)
    st = stream_handle(dev)
    blk = a.block
    body = 65536

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.iters  # us per launch

    def place(data, where):
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        if where == "hbm":
            return t.to(dev)
        p = torch.empty(t.numel(), dtype=torch.uint8, pin_memory=True)
        p.copy_(t)
        return p

    def empty(n, where):
        if where == "hbm":
            return torch.zeros(n, dtype=torch.uint8, device=dev)
        return torch.zeros(n, dtype=torch.uint8, pin_memory=True)

    for kind in a.kinds.split(","):
        raws = [text_body(body, 7 + k) if kind == "text" else b"x" * body if kind == "const" else os.urandom(body)
                for k in range(a.bodies)]
        raw = b"".join(raws)
        total = len(raw)
        npieces = total // blk
        # host-encoded pieces (headerless: varint preamble stripped), the
        # shape the RPC path's host cut hands the piece decoder
        comps = []
        for i in range(npieces):
            c = native.snappy_compress(raw[i * blk:(i + 1) * blk])
            h = 1
            while c[h - 1] & 0x80:
                h += 1
            comps.append(c[h:])
        packed = b"".join(comps)
        ratio = total / max(1, len(packed))
        for src_at in ([] if a.compress_only else a.places.split(",")):
            for dst_at in a.places.split(","):
                cin = place(packed, src_at)
                out = empty(total, dst_at)
                rec, pos = b"", 0
                for i, c in enumerate(comps):
                    rec += struct.pack("<QQII", cin.data_ptr() + pos, out.data_ptr() + i * blk, len(c), blk)
                    pos += len(c)
                pieces = torch.frombuffer(bytearray(rec), dtype=torch.uint8).to(dev)
                err = torch.zeros(npieces, dtype=torch.int32, device=dev)
                for impl in ("parallel", "serial"):
                    fn = (native.gpu.snappy_decompress_pieces_launch if impl == "parallel"
                          else native.gpu.snappy_decompress_pieces_serial_launch)
                    out.zero_()
                    us = timed(lambda: fn(pieces.data_ptr(), npieces, 0, blk, err.data_ptr(), st))
                    torch.cuda.synchronize()
                    ok = int(err.abs().sum().item()) == 0 and bytes(out.cpu().numpy().tobytes()) == raw
                    phases = None
                    if impl == "parallel":
                        stamps = torch.zeros(16, dtype=torch.int64, device=dev)
                        native.gpu.snappy_decompress_pieces_stamped_launch(pieces.data_ptr(), npieces, 0, blk,
                                                                           err.data_ptr(), stamps.data_ptr(), st)
                        torch.cuda.synchronize()
                        t = stamps.cpu().tolist()
                        # shader-clock cycles per phase of block 0
                        phases = {k: t[i + 1] - t[i] for i, k in
                                  enumerate(("stage", "parse_map", "resolve", "gather"))}
                        phases.update({"parse_decode": t[5], "parse_chain": t[6], "parse_fill": t[7],
                                       "parse_iters": t[9]})
                    print(json.dumps({"kernel": "snappy_decompress_pieces", "impl": impl, "body": kind,
                                      "block0_phase_cycles": phases,
                                      "src": src_at, "dst": dst_at, "pieces": npieces, "bytes_out": total,
                                      "ratio": round(ratio, 3), "us_per_launch": round(us, 1),
                                      "GBps_out": round(total / us / 1e3, 2), "verified": ok,
                                      "errs": sorted(set(err.cpu().tolist()))}), flush=True)
        cap = (int(native.gpu.snappy_max_compressed_length(blk)) + 15) & ~15
        scratch = torch.empty(npieces * int(native.gpu.snappy_compress_scratch_per_block()), dtype=torch.uint8,
                              device=dev)
        meta = torch.zeros(2 * npieces, dtype=torch.int32, device=dev)
        for src_at in a.places.split(","):
            for dst_at in a.places.split(","):
                rin = place(raw, src_at)
                slots = empty(npieces * cap, dst_at)
                cj = []
                for i in range(npieces):
                    cj += [rin.data_ptr() + i * blk, slots.data_ptr() + i * cap, blk, cap]
                cj_dev = torch.tensor(cj, dtype=torch.int64, device=dev)
                us = timed(lambda: native.gpu.snappy_compress_launch(cj_dev.data_ptr(), npieces, blk,
                                                                     scratch.data_ptr(), meta.data_ptr(),
                                                                     meta.data_ptr() + 4 * npieces, st))
                torch.cuda.synchronize()
                lens = meta[:npieces].cpu().tolist()
                errs = meta[npieces:].cpu().tolist()
                sl = slots.cpu().numpy().tobytes()
                ok = not any(errs) and all(
                    native.snappy_uncompress(sl[i * cap:i * cap + lens[i]]) == raw[i * blk:(i + 1) * blk]
                    for i in range(0, npieces, 7))
                stamps = torch.zeros(16, dtype=torch.int64, device=dev)
                native.gpu.snappy_compress_stamped_launch(cj_dev.data_ptr(), npieces, blk, scratch.data_ptr(),
                                                          meta.data_ptr(), meta.data_ptr() + 4 * npieces,
                                                          stamps.data_ptr(), st)
                torch.cuda.synchronize()
                t = stamps.cpu().tolist()
                # shader-clock cycles per phase of block 0
                names = ("stage", "first_pos", "match", "write")
                phases = {k: t[i + 1] - t[i] for i, k in enumerate(names)}
                phases.update({"first_pos_atomics": t[8] - t[1], "walk_iters_wave": t[5], "walk_iters_lane_mean": round(t[6] / 64, 1),
                               "walk_matches_lane_mean": round(t[7] / 64, 1)})
                print(json.dumps({"kernel": "snappy_compress", "body": kind, "flags": a.flag, "src": src_at, "dst": dst_at,
                                  "block0_phase_cycles": phases,
                                  "blocks": npieces, "bytes_in": total,
                                  "ratio": round(total / max(1, sum(lens)), 3),
                                  "host_ratio": round(ratio, 3), "us_per_launch": round(us, 1),
                                  "GBps_in": round(total / us / 1e3, 2), "verified": ok}), flush=True)


if __name__ == "__main__":
    main()
