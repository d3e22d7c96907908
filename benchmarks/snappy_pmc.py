"""Small driver for rocprofv3 --pmc runs over the snappy kernels only:
512 x 64 KiB blocks of the mixed corpus, one decompress and one compress
launch (after a warm-up launch of each)."""
import random
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from brpc_amd import native  # noqa: E402
from brpc_amd.ops import snappy_compress, snappy_decompress  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    rnd = random.Random(5)
    base = bytearray()
    while len(base) < 65536:
        base += bytes(rnd.getrandbits(8) for _ in range(24)) if rnd.random() < 0.5 else base[-64:][:32] or b"x" * 32
    base = bytes(base[:65536])
    n = 512
    raw = b"".join(base[i:] + base[:i] for i in range(0, n * 13, 13))
    comps = [native.snappy_compress(raw[i * 65536:(i + 1) * 65536]) for i in range(n)]
    packed = b"".join(comps)
    offs, pos = [], 0
    for c in comps:
        offs.append(pos)
        pos += len(c)
    d = torch.frombuffer(bytearray(packed), dtype=torch.uint8).to(dev)
    raw_dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)
    for _ in range(2):
        out = snappy_decompress(d, offs, [len(c) for c in comps], [65536] * n)
        gp, go, gs, gr = snappy_compress(raw_dev)
    torch.cuda.synchronize()
    assert torch.equal(out, raw_dev)
    print("ok", len(packed), sum(gs))


if __name__ == "__main__":
    main()
