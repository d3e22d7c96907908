"""Packed numeric fields decoded where they already live (HBM -> HBM):
gpu::DeviceDecodePackedRuns over one run of N bytes, timed on the host
around the blocking call (the codec batch's launch, two kernels and the
event) and reported as input GB/s and HBM GB/s (both kernel passes read the
run; the decoded array is written once). Prints one JSON line per size.

  python benchmarks/device_packed_bw.py [--sizes-mb 1,16,64] [--iters 20]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def varints(wire):
    wire = wire.astype(np.uint64)
    nbytes = np.ones(wire.shape, dtype=np.int64)
    for k in range(1, 10):
        nbytes += (wire >> np.uint64(7 * k)) > 0
    start = np.cumsum(nbytes) - nbytes
    out = np.zeros(int(nbytes.sum()), dtype=np.uint8)
    for k in range(10):
        m = nbytes > k
        byte = ((wire[m] >> np.uint64(7 * k)) & np.uint64(0x7F)).astype(np.uint8)
        byte |= np.where(nbytes[m] > k + 1, 0x80, 0).astype(np.uint8)
        out[start[m] + k] = byte
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="1,16,64")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shapes", default="ids,u64", help="ids: int32 ids < 2^14 (2-byte varints); u64: full-width")
    args = ap.parse_args()
    from brpc_amd import native
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(1)
    for shape in args.shapes.split(","):
        kind, esize, per = (0, 4, 2) if shape == "ids" else (4, 8, 10)
        for mb in [float(x) for x in args.sizes_mb.split(",")]:
            n = int(mb * (1 << 20)) // per
            vals = rng.integers(1 << 7, 1 << 14, n) if shape == "ids" else \
                rng.integers(1 << 63, (1 << 64) - 1, n, dtype=np.uint64)
            wire = varints(vals)
            src = torch.from_numpy(wire).to(dev)
            dst = torch.empty(n * esize, dtype=torch.uint8, device=dev)
            call = lambda: native.gpu.device_decode_packed([src.data_ptr()], [len(wire)], [kind],
                                                           [dst.data_ptr()], 0)
            torch.cuda.synchronize()  # the upload runs on torch's stream, the decoder on ours
            [(count, code)] = call()
            assert code == 0 and count == n, (count, code, n)
            got = dst.view(torch.int32 if kind == 0 else torch.int64)[:16].cpu().numpy()
            want = vals[:16].astype(np.int32) if kind == 0 else vals[:16].view(np.int64)
            assert np.array_equal(got, want)
            for _ in range(3):
                call()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.iters):
                call()
            dt = (time.perf_counter() - t0) / args.iters
            hbm = 2 * len(wire) + n * esize
            print(json.dumps({"shape": shape, "run_bytes": len(wire), "elements": n, "us_per_call": round(dt * 1e6, 1),
                              "input_gb_per_s": round(len(wire) / dt / 1e9, 1),
                              "hbm_gb_per_s": round(hbm / dt / 1e9, 1)}), flush=True)
    print(json.dumps({"device_codec_stats": native.gpu.device_codec_stats()}))


if __name__ == "__main__":
    main()
