"""Data-parallel compressor on small inputs with per-position state dumps (debug aid)."""
import sys
import torch
sys.path.insert(0, ".")
from brpc_amd import native
from brpc_amd.ops._common import stream_handle

native.set_flag("gpu_snappy_compress_pj", "true")
dev = torch.device("cuda", 0)
for data in [b"abcdefgh" * 3]:
    n = len(data)
    src = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    for max_ulen in (24, 40):
        cap = 256
        out = torch.zeros(cap, dtype=torch.uint8, device=dev)
        jobs = torch.tensor([src.data_ptr(), out.data_ptr(), n, cap], dtype=torch.int64, device=dev)
        meta = torch.zeros(2, dtype=torch.int32, device=dev)
        stamps = torch.zeros(320, dtype=torch.int64, device=dev)
        stamps[7] = 0xDEB6
        torch.cuda.synchronize()
        native.gpu.snappy_compress_stamped_launch(jobs.data_ptr(), 1, max_ulen, 0, meta.data_ptr(),
                                                  meta.data_ptr() + 4, stamps.data_ptr(), stream_handle(dev))
        torch.cuda.synchronize()
        m = meta.cpu().tolist()
        o = out[:m[0]].cpu().numpy().tobytes()
        st = stamps.cpu().tolist()
        print("max_ulen", max_ulen, "n", n, "len/err", m, o.hex()[:60], flush=True)
        print("   stored", [(x & 0xFFFF, (x >> 16) & 0xFFFF, (x >> 32) & 0xFFFF) for x in st[240:240 + n]])
        for base, name in ((16, "after L"),):
            print("  ", name, [(x & 0xFF, (x >> 8) & 0xFFFF, (x >> 24) & 0xFF, (x >> 32) & 0xFFFF)
                               for x in st[base:base + min(n, 12)]], flush=True)
