"""Throughput of the GPU JSON structural index (gpu/json_kernels.hip) on
json.dumps documents of several sizes; buffers are preallocated so the timed
loop is the five launches only. Prints one line per size."""
import json
import random
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from brpc_amd.native import native  # noqa: E402
from brpc_amd.ops._common import stream_handle  # noqa: E402


def doc(rnd, depth=0):
    k = rnd.random()
    if depth > 3 or k < 0.35:
        return rnd.choice([rnd.randint(-10**9, 10**9), rnd.random(), True, None,
                           "".join(rnd.choice('abcdefgh "\\/xyz') for _ in range(rnd.randint(0, 24)))])
    if k < 0.6:
        return [doc(rnd, depth + 1) for _ in range(rnd.randint(0, 6))]
    return {"key%d" % i: doc(rnd, depth + 1) for i in range(rnd.randint(0, 6))}


def main():
    dev = torch.device("cuda", 0)
    rnd = random.Random(1)
    unit = json.dumps([doc(rnd) for _ in range(2000)]).encode() + b","
    for mib in (1, 16, 256):
        n = mib << 20
        data = (unit * (n // len(unit) + 1))[:n]
        buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
        out = torch.empty(n // 2, dtype=torch.int32, device=dev)
        meta = torch.zeros(2, dtype=torch.int64, device=dev)
        scratch = torch.empty(native.gpu.json_index_scratch_bytes(n), dtype=torch.uint8, device=dev)
        s = stream_handle(dev)

        def run():
            native.gpu.json_index_launch(buf.data_ptr(), n, out.data_ptr(), out.numel(), meta.data_ptr(),
                                         meta.data_ptr() + 8, scratch.data_ptr(), s)

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        iters = max(5, 2000 // mib)
        t0 = time.perf_counter()
        for _ in range(iters):
            run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / iters
        count, err = meta.tolist()
        print("json_index %4d MiB: %8.1f us  %7.1f GB/s  positions=%d err=%d" % (mib, dt * 1e6, n / dt / 1e9, count,
                                                                             err), flush=True)


if __name__ == "__main__":
    main()
