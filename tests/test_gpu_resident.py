"""Resident copy worker (gpu/kernels.hip resident_copy_kernel behind
gpu/copy_engine.cc with -copy_engine_resident): batches go through a pinned
ring to a persistent kernel instead of a launch each.

Everything runs in a child process with its own time limit (a persistent
kernel that failed to exit would otherwise hold the test runner):
  * copies and CRC32C (per segment and folded per message, checksum-only
    segments) of random unaligned segments from HBM and pinned memory,
    issued from several threads at once, against torch / the host CRC;
  * an echo press over device attachments and the GPU handler through it;
  * instances exit when idle and are relaunched by the next batch."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

_PROBE = r"""
import json, random, sys, threading, time
sys.path.insert(0, sys.argv[1])
import torch
from brpc_amd import native
native.set_flag("copy_engine_resident", "true")
dev = torch.device("cuda:0")
rnd = random.Random(7)

src = torch.randint(0, 256, (8 << 20,), dtype=torch.uint8, device=dev)
pin = torch.randint(0, 256, (4 << 20,), dtype=torch.uint8).pin_memory()
torch.cuda.synchronize()  # randint runs on torch's stream, the copy engine on its own
errors = []

def worker(seed, rounds):
    r = random.Random(seed)
    for _ in range(rounds):
        n = r.randint(1, 40)
        srcs, dsts, lens, views = [], [], [], []
        out = torch.empty(9 << 20, dtype=torch.uint8, device=dev)
        pos = 0
        for i in range(n):
            ln = r.choice([1, 7, 100, 4096, 16384, 65536, 65537, 200000])
            from_pin = r.random() < 0.3
            base = pin if from_pin else src
            off = r.randint(0, base.numel() - ln)
            srcs.append(base.data_ptr() + off)
            dsts.append(out.data_ptr() + pos)
            lens.append(ln)
            views.append((base, off, ln, pos))
            pos += ln + r.randint(0, 3)
        with_crc = r.random() < 0.7
        fold = with_crc and r.random() < 0.4
        crcs = native.gpu.engine_copy(srcs, dsts, lens, 0, with_crc, fold)
        torch.cuda.synchronize()
        for (base, off, ln, p) in views:
            a = base[off:off + ln].to(dev)
            if not torch.equal(out[p:p + ln], a):
                errors.append("copy mismatch len=%d" % ln)
        if with_crc:
            blobs = [bytes(base[off:off + ln].cpu().numpy().tobytes()) for (base, off, ln, p) in views]
            want = [native.crc32c(b"".join(blobs))] if fold else [native.crc32c(b) for b in blobs]
            if list(crcs) != want:
                errors.append("crc mismatch fold=%s n=%d" % (fold, n))

ths = [threading.Thread(target=worker, args=(s, 25)) for s in range(6)]
for t in ths: t.start()
for t in ths: t.join()
# checksum-only segments (dst 0)
blob = src[:300000]
c = native.gpu.engine_copy([blob.data_ptr()], [0], [300000], 0, True, False)
if c[0] != native.crc32c(bytes(blob.cpu().numpy().tobytes())):
    errors.append("crc-only mismatch")
s0 = native.gpu.resident_stats()
time.sleep(0.05)  # instances exit when idle; the next batch relaunches one
c2 = native.gpu.engine_copy([blob.data_ptr()], [0], [300000], 0, True, False)
if c2 != c:
    errors.append("crc after idle exit mismatch")
s1 = native.gpu.resident_stats()
# the RPC paths over it
from brpc_amd.models import start_echo_server
srv = start_echo_server("127.0.0.1:0", gpu_device=0)
res = {}
for name, opts in (("lend", {"device_attachment": True}), ("handler", {"gpu_process": True})):
    p = native.Press(dict({"server": srv.address, "concurrency": 32, "attachment_size": 65536, "gpu_device": 0,
                           "check_echo": True}, **opts))
    p.run_requests(3000)
    st = p.stats()
    res[name] = [st["success"], st["error"]]
srv.stop()
s2 = native.gpu.resident_stats()
print(json.dumps({"errors": errors[:5], "nerr": len(errors), "s0": s0, "s1": s1, "s2": s2, "rpc": res}))
"""


def test_resident_copy_worker_numerics_rpc_and_idle_exit():
    r = subprocess.run(["timeout", "-k", "5", "150", sys.executable, "-c", _PROBE, ROOT], capture_output=True,
                       text=True, timeout=170)
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    import json
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["nerr"] == 0, out["errors"]
    assert out["s0"]["batches"] > 0 and out["s0"]["launches"] >= 1
    # amortized: many batches per instance
    assert out["s2"]["batches"] > 5 * out["s2"]["launches"], out
    # the idle instance exited and the next batch started a new one
    assert out["s1"]["launches"] > out["s0"]["launches"], out
    assert out["rpc"]["lend"] == [3000, 0] and out["rpc"]["handler"] == [3000, 0], out
