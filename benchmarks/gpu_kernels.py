#!/usr/bin/env python3
"""Throughput of the device data-path kernels (CRC32C, varint codec,
batched copy) on one MI355X, measured with HIP events; prints one JSON line
per kernel. HBM peak for reference: ~6.3 TB/s measured copy."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from brpc_amd.ops import batched_copy, crc32c_batch, crc32c_host, crc32c_packed, varint_decode, varint_encode  # noqa: E402


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters / 1e3  # seconds


def main():
    dev = torch.device("cuda", 0)
    sizes = [int(x) for x in os.environ.get("SIZES", str(1 << 28)).split(",")]
    for n in sizes:
        buf = torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev)
        for impl in ("mfma", "lds"):
            t = timeit(lambda: crc32c_batch([buf], impl=impl))
            print(json.dumps({"kernel": "crc32c_" + impl, "bytes": n, "sec": t, "GBps": n / t / 1e9}))
        small = buf[: 1 << 24]
        ok = int(crc32c_batch([small])[0]) == crc32c_host(small.cpu().numpy().tobytes())
        print(json.dumps({"kernel": "crc32c_verify_16MiB", "verified": ok}))
        offs = torch.arange(0, n + 1, 65536, dtype=torch.int64, device=dev)
        t = timeit(lambda: crc32c_packed(buf, offs))
        print(json.dumps({"kernel": "crc32c_packed_64KiB", "messages": offs.numel() - 1, "bytes": n, "sec": t,
                          "GBps": n / t / 1e9}))
        # many 64 KiB messages in one launch set (the RPC batch case)
        msgs = [buf[i * 65536:(i + 1) * 65536] for i in range(min(4096, n // 65536))]
        if msgs:
            t = timeit(lambda: crc32c_batch(msgs))
            tot = 65536 * len(msgs)
            print(json.dumps({"kernel": "crc32c_batch_64KiB", "messages": len(msgs), "bytes": tot, "sec": t,
                              "GBps": tot / t / 1e9}))
        dst = torch.empty_like(buf)
        t = timeit(lambda: batched_copy([buf], [dst]))
        print(json.dumps({"kernel": "batched_copy", "bytes": n, "sec": t, "GBps": 2 * n / t / 1e9}))
        t = timeit(lambda: dst.copy_(buf))
        print(json.dumps({"kernel": "torch_copy_reference", "bytes": n, "sec": t, "GBps": 2 * n / t / 1e9}))
        nv = n // 8
        vals = torch.randint(-(2 ** 62), 2 ** 62, (nv,), dtype=torch.int64, device=dev) >> torch.randint(
            0, 62, (nv,), dtype=torch.int64, device=dev)
        enc = varint_encode(vals)
        t = timeit(lambda: varint_encode(vals), iters=5)
        print(json.dumps({"kernel": "varint_encode", "values": nv, "bytes_out": enc.numel(), "sec": t,
                          "Mvalues_per_s": nv / t / 1e6, "GBps_in": nv * 8 / t / 1e9}))
        t = timeit(lambda: varint_decode(enc), iters=5)
        ok = bool(torch.equal(varint_decode(enc), vals))
        print(json.dumps({"kernel": "varint_decode", "values": nv, "bytes_in": enc.numel(), "sec": t,
                          "Mvalues_per_s": nv / t / 1e6, "verified": ok}))
        del buf, dst, vals, enc
        torch.cuda.empty_cache()
    # snappy decompression: 2048 blocks x 64 KiB of mixed (~2:1) data
    from brpc_amd import native
    from brpc_amd.ops import snappy_decompress
    import random
    rnd = random.Random(5)
    blk = bytearray()
    while len(blk) < 65536:
        blk += bytes(rnd.getrandbits(8) for _ in range(24)) if rnd.random() < 0.5 else blk[-64:][:32] or b"x" * 32
    blk = bytes(blk[:65536])
    comps = [native.snappy_compress(blk[i:] + blk[:i]) for i in range(0, 2048 * 13, 13)]
    packed = b"".join(comps)
    offs, pos = [], 0
    for c in comps:
        offs.append(pos)
        pos += len(c)
    d = torch.frombuffer(bytearray(packed), dtype=torch.uint8).to(dev)
    sizes = [len(c) for c in comps]
    outs = [65536] * len(comps)
    out = torch.empty(65536 * len(comps), dtype=torch.uint8, device=dev)
    res = snappy_decompress(d, offs, sizes, outs, out=out)
    ok = bytes(res[:65536].cpu().numpy().tobytes()) == blk
    t = timeit(lambda: snappy_decompress(d, offs, sizes, outs, out=out), iters=5)
    nout = 65536 * len(comps)
    print(json.dumps({"kernel": "snappy_decompress_64KiB_blocks", "blocks": len(comps), "bytes_in": len(packed),
                      "bytes_out": nout, "sec": t, "GBps_out": nout / t / 1e9, "verified": ok}))


if __name__ == "__main__":
    main()
