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
        from brpc_amd.ops import batched_copy_crc32c
        for mfma, name in ((True, "copy_crc32c_fused"), (False, "copy_crc32c_fused_table")):
            ok = int(batched_copy_crc32c([small], [dst[: small.numel()]], mfma=mfma)[0]) == crc32c_host(
                small.cpu().numpy().tobytes())
            t = timeit(lambda: batched_copy_crc32c([buf], [dst], mfma=mfma))
            print(json.dumps({"kernel": name, "bytes": n, "sec": t, "GBps_read": n / t / 1e9,
                              "GBps_rw": 2 * n / t / 1e9, "verified": ok}))
            # the verified pull's launch shapes: 32 x 1 MiB and 32 x 64 KiB
            for seg in (1 << 20, 65536):
                k = min(32, n // seg)
                ss = [buf[i * seg:(i + 1) * seg] for i in range(k)]
                dd = [dst[i * seg:(i + 1) * seg] for i in range(k)]
                t = timeit(lambda: batched_copy_crc32c(ss, dd, mfma=mfma))
                print(json.dumps({"kernel": "%s_%dx%dKiB" % (name, k, seg >> 10), "bytes": k * seg, "sec": t,
                                  "GBps_read": k * seg / t / 1e9}))
        # the transport's per-tick pull: 64 x 64 KiB payloads in one launch set
        nb = min(64, n // 65536)
        pulls_s = [buf[i * 65536:(i + 1) * 65536] for i in range(nb)]
        pulls_d = [dst[i * 65536:(i + 1) * 65536] for i in range(nb)]
        t = timeit(lambda: batched_copy(pulls_s, pulls_d))
        print(json.dumps({"kernel": "pull_batch_64x64KiB", "bytes": nb * 65536, "sec": t,
                          "GBps_rw": 2 * nb * 65536 / t / 1e9}))
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
    # protobuf wire scan: 4M RpcMeta-sized messages (tag/varint/len walk)
    from brpc_amd.ops import pb_scan
    import random as _r
    rnd0 = _r.Random(11)

    def _vi(v):
        out = bytearray()
        while v >= 0x80:
            out.append((v & 0x7F) | 0x80)
            v >>= 7
        out.append(v)
        return bytes(out)

    tmpl = []
    for _ in range(1024):  # RpcMeta-like: request{service,method,log_id}, correlation_id, attachment_size
        req = b"\x0a" + _vi(20) + b"example.EchoService_" + b"\x12\x04Echo" + b"\x18" + _vi(rnd0.getrandbits(40))
        tmpl.append(b"\x0a" + _vi(len(req)) + req + b"\x20" + _vi(rnd0.getrandbits(50)) + b"\x28" + _vi(rnd0.randrange(1 << 17)))
    nmsg = 1 << 22
    lens = torch.tensor([len(m) for m in tmpl], dtype=torch.int64)
    t_bytes = torch.frombuffer(bytearray(b"".join(tmpl)), dtype=torch.uint8)
    reps = nmsg // len(tmpl)
    pbbuf = t_bytes.repeat(reps).to(dev)
    pboffs = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(lens.repeat(reps), 0)]).to(dev)
    fields, nf = pb_scan(pbbuf, pboffs, 8)
    ok = bool((nf == 3).all().item())
    t = timeit(lambda: pb_scan(pbbuf, pboffs, 8), iters=10)
    print(json.dumps({"kernel": "pb_scan", "messages": nmsg, "bytes": pbbuf.numel(), "sec": t,
                      "Mmsgs_per_s": nmsg / t / 1e6, "GBps_in": pbbuf.numel() / t / 1e9, "verified": ok}))
    del pbbuf, pboffs, fields, nf
    torch.cuda.empty_cache()

    # snappy: 128 MiB of mixed (~2:1) data as 2048 x 64 KiB, 4096 x 32 KiB and
    # 32768 x 4 KiB (the RPC offload's block)
    # blocks. "sec" is kernel time only (CUDA events around launches with the
    # job tables already on the device); the python wrappers add host work.
    from brpc_amd import native
    from brpc_amd.ops import snappy_compress, snappy_decompress
    from brpc_amd.ops._common import stream_handle
    import random
    rnd = random.Random(5)
    base = bytearray()
    while len(base) < 65536:
        base += bytes(rnd.getrandbits(8) for _ in range(24)) if rnd.random() < 0.5 else base[-64:][:32] or b"x" * 32
    base = bytes(base[:65536])
    total = 128 << 20
    raw = b"".join(base[i:] + base[:i] for i in range(0, (total // 65536) * 13, 13))
    raw_dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)

    def kernel_time(fn, iters=10):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / 1e3 / iters

    for block in (65536, 32768, 4096):
        n = total // block
        # host codec blocks -> device decompression
        comps = [native.snappy_compress(raw[i * block:(i + 1) * block]) for i in range(n)]
        packed = b"".join(comps)
        offs, pos = [], 0
        for c in comps:
            offs.append(pos)
            pos += len(c)
        d = torch.frombuffer(bytearray(packed), dtype=torch.uint8).to(dev)
        out = torch.empty(total, dtype=torch.uint8, device=dev)
        res = snappy_decompress(d, offs, [len(c) for c in comps], [block] * n, out=out)
        ok = bool(torch.equal(res, raw_dev))
        jobs = []
        for i, c in enumerate(comps):
            jobs += [d.data_ptr() + offs[i], out.data_ptr() + i * block, len(c), block]
        jobs_dev = torch.tensor(jobs, dtype=torch.int64, device=dev)
        meta = torch.zeros(2 * n, dtype=torch.int32, device=dev)
        st = stream_handle(dev)
        t = kernel_time(lambda: native.gpu.snappy_decompress_launch(jobs_dev.data_ptr(), n, block, meta.data_ptr(),
                                                                    meta.data_ptr() + 4 * n, st))
        print(json.dumps({"kernel": "snappy_decompress", "block": block, "blocks": n, "bytes_in": len(packed),
                          "bytes_out": total, "sec": t, "GBps_out": total / t / 1e9, "verified": ok}))
        # device compression -> host + device decompression checks
        gp, goffs, gsizes, graw = snappy_compress(raw_dev, block=block)
        host = gp.cpu().numpy().tobytes()
        ok_host = all(native.snappy_uncompress(host[o:o + s]) == raw[i * block:(i + 1) * block]
                      for i, (o, s) in enumerate(zip(goffs[:64], gsizes[:64])))
        back = snappy_decompress(gp, goffs, gsizes, graw)
        ok_dev = bool(torch.equal(back, raw_dev))
        cap = (int(native.gpu.snappy_max_compressed_length(block)) + 15) & ~15
        slots = torch.empty(n * cap, dtype=torch.uint8, device=dev)
        scratch = torch.empty(n * int(native.gpu.snappy_compress_scratch_per_block()), dtype=torch.uint8, device=dev)
        cj = []
        for i in range(n):
            cj += [raw_dev.data_ptr() + i * block, slots.data_ptr() + i * cap, block, cap]
        cj_dev = torch.tensor(cj, dtype=torch.int64, device=dev)
        t = kernel_time(lambda: native.gpu.snappy_compress_launch(cj_dev.data_ptr(), n, block, scratch.data_ptr(),
                                                                  meta.data_ptr(), meta.data_ptr() + 4 * n, st))
        print(json.dumps({"kernel": "snappy_compress", "block": block, "blocks": n, "bytes_in": total,
                          "bytes_out": int(sum(gsizes)), "host_codec_bytes_out": len(packed), "sec": t,
                          "GBps_in": total / t / 1e9, "verified_host_decode": ok_host, "verified_gpu_decode": ok_dev}))
        del d, out, jobs_dev, slots, scratch, cj_dev, gp, back
        torch.cuda.empty_cache()

if __name__ == "__main__":
    main()
