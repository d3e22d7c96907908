"""Numerics of the gfx950 kernels against host references (CPU crc32c via
SSE4.2, pure-python varint codec), plus the device-payload echo path."""
import os
import random
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from brpc_amd import native
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    assert native.gpu.device_count() > 0, "native runtime sees no HIP device"
    assert native.gpu.device_arch(0) == "gfx950"
    return torch.device("cuda", 0)


@pytest.mark.parametrize("n", [0, 1, 7, 63, 64, 65, 1000, 16383, 16384, 16385, 65536, 100003, 1 << 20, (1 << 24) + 5])
def test_crc32c_matches_host(dev, n):
    from brpc_amd.ops import crc32c, crc32c_host
    g = torch.Generator().manual_seed(n)
    host = torch.randint(0, 256, (n,), dtype=torch.uint8, generator=g)
    want = crc32c_host(host.numpy().tobytes())
    d = host.to(dev)
    assert crc32c(d, impl="mfma") == want
    assert crc32c(d, impl="lds") == want


def test_crc32c_single_bits(dev):
    """Every bit of a 2 KiB group exercises one A-matrix column of the MFMA
    kernel: a wrong fragment mapping shows up as a mismatch here."""
    from brpc_amd.ops import crc32c_batch, crc32c_host
    base = torch.zeros(4096, dtype=torch.uint8)
    bufs = []
    for bit in range(0, 4096 * 8, 61):
        b = base.clone()
        b[bit // 8] = 1 << (bit % 8)
        bufs.append(b)
    got = crc32c_batch([b.to(dev) for b in bufs]).tolist()
    want = [crc32c_host(b.numpy().tobytes()) for b in bufs]
    assert got == want


def test_crc32c_packed(dev):
    from brpc_amd.ops import crc32c_host, crc32c_packed
    sizes = [0, 1, 100, 65536, 65537, 3, 200000, 16]
    buf = torch.randint(0, 256, (sum(sizes),), dtype=torch.uint8, device=dev)
    offs = [0]
    for s in sizes:
        offs.append(offs[-1] + s)
    got = crc32c_packed(buf, torch.tensor(offs, dtype=torch.int64, device=dev)).tolist()
    hb = buf.cpu().numpy().tobytes()
    assert got == [crc32c_host(hb[offs[i]:offs[i + 1]]) for i in range(len(sizes))]


def test_crc32c_known_vector(dev):
    from brpc_amd.ops import crc32c
    t = torch.tensor(list(b"123456789"), dtype=torch.uint8, device=dev)
    assert crc32c(t) == 0xE3069283


def test_crc32c_unaligned_views_and_batch(dev):
    from brpc_amd.ops import crc32c_batch, crc32c_host
    base = torch.randint(0, 256, (300000,), dtype=torch.uint8, device=dev)
    views = [base[o:o + l] for o, l in [(1, 5000), (3, 70000), (17, 16384), (0, 1), (5, 0)]] * 10  # 50 > 32 inline
    want = [crc32c_host(v.cpu().numpy().tobytes()) for v in views]
    assert crc32c_batch(views).tolist() == want
    assert crc32c_batch(views, impl="lds").tolist() == want


def test_varint_roundtrip(dev):
    from brpc_amd.ops import varint_decode, varint_encode, varint_encode_host
    rnd = random.Random(1)
    vals = [0, 1, 127, 128, 300, 2**31 - 1, -1, -(2**63), 2**63 - 1] + \
        [rnd.randrange(-(2**63), 2**63) >> rnd.randrange(0, 63) for _ in range(20000)]
    t = torch.tensor(vals, dtype=torch.int64, device=dev)
    enc = varint_encode(t)
    assert enc.cpu().numpy().tobytes() == varint_encode_host(vals)
    dec = varint_decode(enc)
    assert dec.cpu().tolist() == vals


def test_varint_zigzag(dev):
    from brpc_amd.ops import varint_decode, varint_encode, varint_encode_host
    vals = list(range(-5000, 5000, 7))
    t = torch.tensor(vals, dtype=torch.int64, device=dev)
    enc = varint_encode(t, zigzag=True)
    assert enc.cpu().numpy().tobytes() == varint_encode_host(vals, zigzag=True)
    assert varint_decode(enc, zigzag=True).cpu().tolist() == vals


def test_varint_malformed(dev):
    from brpc_amd.ops import varint_decode
    bad = torch.tensor([0x80] * 12 + [0x01], dtype=torch.uint8, device=dev)
    with pytest.raises(ValueError):
        varint_decode(bad)
    trunc = torch.tensor([0x05, 0x80], dtype=torch.uint8, device=dev)
    with pytest.raises(ValueError):
        varint_decode(trunc)


def test_batched_copy(dev):
    from brpc_amd.ops import batched_copy
    srcs = [torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev) for n in (1, 15, 16, 4097, 70000, 1 << 20)]
    dsts = [torch.zeros_like(s) for s in srcs]
    batched_copy(srcs, dsts)
    torch.cuda.synchronize()
    for s, d in zip(srcs, dsts):
        assert torch.equal(s, d)
    # unaligned
    big = torch.randint(0, 256, (10000,), dtype=torch.uint8, device=dev)
    out = torch.zeros(10000, dtype=torch.uint8, device=dev)
    batched_copy([big[3:9003]], [out[5:9005]])
    torch.cuda.synchronize()
    assert torch.equal(big[3:9003], out[5:9005])


def test_device_payload_echo(dev):
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    try:
        p = native.Press({"server": s.address, "concurrency": 8, "attachment_size": 65536,
                          "device_attachment": True, "gpu_device": 0, "check_echo": True})
        p.run_requests(500)
        st = p.stats()
        assert st["success"] == 500 and st["error"] == 0, st
    finally:
        s.stop()


def test_device_payload_uses_xgmi_in_process(dev):
    """Same-process peers: the hello maps the local arena; payloads skip TCP."""
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    try:
        before = native.gpu.xgmi_stats()
        p = native.Press({"server": s.address, "concurrency": 4, "attachment_size": 1 << 20,
                          "device_attachment": True, "gpu_device": 0, "check_echo": True})
        p.run_requests(200)
        st = p.stats()
        assert st["success"] == 200 and st["error"] == 0, st
        after = native.gpu.xgmi_stats()
        # the first call(s) of a connection are staged through host while the
        # hello is in flight; everything after moves over the device arena
        assert after["sent_payloads"] - before["sent_payloads"] >= 100, (before, after)
        assert after["recv_payloads"] - before["recv_payloads"] >= 100, (before, after)
        assert after["crc_failures"] == before["crc_failures"]
    finally:
        s.stop()


_SERVER_SCRIPT = r"""
import sys, torch
from brpc_amd.models import start_echo_server
s = start_echo_server("127.0.0.1:0", gpu_device=0)
print(s.port, flush=True)
sys.stdin.read()
s.stop()
"""


def test_device_payload_xgmi_cross_process(dev):
    """Two processes on one GPU: IPC-mapped arenas + shm release tables."""
    import os
    import subprocess
    import sys
    from brpc_amd import native
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=repo + os.pathsep + os.environ.get("PYTHONPATH", ""))
    srv = subprocess.Popen([sys.executable, "-c", _SERVER_SCRIPT], stdin=subprocess.PIPE,
                           stdout=subprocess.PIPE, env=env, text=True)
    try:
        port = int(srv.stdout.readline())
        before = native.gpu.xgmi_stats()
        p = native.Press({"server": "127.0.0.1:%d" % port, "concurrency": 4, "attachment_size": 1 << 20,
                          "device_attachment": True, "gpu_device": 0, "check_echo": True})
        p.run_requests(200)
        st = p.stats()
        assert st["success"] == 200 and st["error"] == 0, st
        after = native.gpu.xgmi_stats()
        assert after["sent_payloads"] - before["sent_payloads"] >= 100, (before, after)
        assert after["recv_payloads"] - before["recv_payloads"] >= 100, (before, after)
    finally:
        srv.stdin.close()
        srv.wait(timeout=60)


def _drain_lent(native, timeout_s=5.0):
    import time
    deadline = time.time() + timeout_s
    while time.time() < deadline:
        native.gpu.reap_lent()
        st = native.gpu.xgmi_stats()
        if st["lent_outstanding"] == 0:
            return st
        time.sleep(0.05)
    return native.gpu.xgmi_stats()


def test_device_payload_zero_copy_lending(dev):
    """Arena-resident attachments are lent (no sender-side copy), pulled once
    per hop by the batched copy engine, and every lend is released."""
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    try:
        before = native.gpu.xgmi_stats()
        p = native.Press({"server": s.address, "concurrency": 32, "attachment_size": 65536,
                          "device_attachment": True, "gpu_device": 0, "check_echo": True})
        p.run_requests(2000)
        st = p.stats()
        assert st["success"] == 2000 and st["error"] == 0, st
        after = _drain_lent(native)
        assert after["lent_outstanding"] == 0, after
        assert after["copied_into_arena"] == before["copied_into_arena"], (before, after)
        assert after["ring_full_fallbacks"] == before["ring_full_fallbacks"], (before, after)
        pulls = after["copy_segments"] - before["copy_segments"]
        launches = after["copy_launches"] - before["copy_launches"]
        assert pulls >= 3000, (before, after)
        # concurrent pulls are combined into shared launches
        assert launches < pulls, (pulls, launches)
        pool = native.gpu.hbm_pool_stats(0)
        assert pool["fallback_allocs"] == 0, pool
        assert pool["pinned_blocks_in_use"], pool
    finally:
        s.stop()


def test_device_payload_released_on_reject(dev):
    """ELIMIT rejections happen before the server looks at the attachment:
    the lent HBM blocks must still come back (baidu_std early
    reject paths)."""
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0", gpu_device=0, max_concurrency=1)
    try:
        before = native.gpu.xgmi_stats()
        p = native.Press({"server": s.address, "concurrency": 16, "attachment_size": 65536,
                          "device_attachment": True, "gpu_device": 0, "max_retry": 0})
        p.run_requests(1000)
        st = p.stats()
        assert st["error"] > 0, st  # some were rejected with ELIMIT
        after = _drain_lent(native)
        assert after["lent_outstanding"] == 0, after
        assert after["released_unconsumed"] > before["released_unconsumed"], (before, after)
        assert after["ring_full_fallbacks"] == before["ring_full_fallbacks"], (before, after)
    finally:
        s.stop()


def test_stream_device_chunks_over_xgmi(dev):
    """Streaming RPC with HBM chunks: frames lend the chunk, the receiver
    pulls it in frame order; nothing is staged through host memory."""
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    servers = [start_echo_server("127.0.0.1:0", gpu_device=0) for _ in range(2)]
    try:
        before = native.gpu.xgmi_stats()
        sp = native.StreamPress({"server": ",".join(s.address for s in servers), "chunk_size": 65536,
                                 "chunks_per_step": 16, "device_chunks": True, "gpu_device": 0})
        sp.run_steps(10)
        st = sp.stats()
        assert st["bytes_acked"] == 2 * 10 * 16 * 65536, st
        sp.close()
        after = _drain_lent(native)
        assert after["recv_payloads"] - before["recv_payloads"] >= 2 * 10 * 16, (before, after)
        assert after["lent_outstanding"] == 0, after
        assert after["copied_into_arena"] == before["copied_into_arena"], (before, after)
    finally:
        for s in servers:
            s.stop()


def test_fanout_device_attachment(dev):
    """ParallelChannel broadcast of one HBM attachment: one lend per peer of
    the same arena block, gathered echoes pulled back."""
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    servers = [start_echo_server("127.0.0.1:0", gpu_device=0) for _ in range(3)]
    try:
        p = native.Press({"server": servers[0].address, "fanout_servers": ",".join(s.address for s in servers),
                          "concurrency": 8, "attachment_size": 65536, "device_attachment": True,
                          "gpu_device": 0, "check_echo": True})
        p.run_requests(300)
        st = p.stats()
        assert st["success"] == 300 and st["error"] == 0, st
        assert [s.echo_calls for s in servers] == [300, 300, 300]
        assert _drain_lent(native)["lent_outstanding"] == 0
    finally:
        for s in servers:
            s.stop()


def test_scatter_device_attachment(dev):
    """TP analog over xGMI: each peer is lent only its (unaligned) slice of
    the HBM attachment and echoes it; the gathered slices are the original."""
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    servers = [start_echo_server("127.0.0.1:0", gpu_device=0) for _ in range(3)]
    try:
        p = native.Press({"server": servers[0].address, "fanout_servers": ",".join(s.address for s in servers),
                          "scatter": True, "concurrency": 8, "attachment_size": 65536 + 7,
                          "device_attachment": True, "gpu_device": 0, "check_echo": True})
        p.run_requests(300)
        st = p.stats()
        assert st["success"] == 300 and st["error"] == 0, st
        assert [s.echo_calls for s in servers] == [300, 300, 300]
        assert _drain_lent(native)["lent_outstanding"] == 0
    finally:
        for s in servers:
            s.stop()


def test_route_device_attachment_by_key(dev):
    """EP analog: keyed calls routed by c_murmurhash to the owning server,
    HBM attachments lent over the transport to whichever server owns the key."""
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    servers = [start_echo_server("127.0.0.1:0", gpu_device=0) for _ in range(4)]
    try:
        p = native.Press({"server": "list://" + ",".join(s.address for s in servers), "lb_policy": "c_murmurhash",
                          "concurrency": 16, "attachment_size": 65536, "device_attachment": True,
                          "gpu_device": 0, "check_echo": True})
        p.run_requests(800)
        st = p.stats()
        assert st["success"] == 800 and st["error"] == 0, st
        calls = [s.echo_calls for s in servers]
        assert sum(calls) == 800 and min(calls) > 0, calls
        assert _drain_lent(native)["lent_outstanding"] == 0
    finally:
        for s in servers:
            s.stop()


def test_stream_relay_chain_device_chunks(dev):
    """PP analog over xGMI: HBM chunks relayed through three servers, each
    hop pulling the chunk and lending it on; acks come back from the tail."""
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    servers = [start_echo_server("127.0.0.1:0", gpu_device=0) for _ in range(3)]
    try:
        before = native.gpu.xgmi_stats()
        sp = native.StreamPress({"server": servers[0].address, "chunk_size": 65536, "chunks_per_step": 16,
                                 "device_chunks": True, "gpu_device": 0,
                                 "relay_chain": ",".join(s.address for s in servers[1:])})
        sp.run_steps(5)
        st = sp.stats()
        assert st["steps"] == 5 and st["bytes_acked"] == 5 * 16 * 65536, st
        sp.close()
        after = _drain_lent(native)
        assert after["lent_outstanding"] == 0, after
        # three hops each pulled every chunk
        assert after["copy_segments"] - before["copy_segments"] >= 3 * 5 * 16, (before, after)
    finally:
        for s in servers:
            s.stop()


@pytest.mark.parametrize("device_attachment", [False, True])
def test_gpu_process_echo_handler(dev, device_attachment):
    """the handler runs the attachment through the fused
    copy+CRC32C kernel — into HBM (lent back over xGMI) when the client has
    a device transport, straight into pinned memory for a TCP client (one
    device round trip); the client checks the bytes and the device CRC
    against the host SSE4.2 CRC32C."""
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    try:
        for size in (1, 4095, 65536 - 16, 300000):
            p = native.Press({"server": s.address, "concurrency": 8, "attachment_size": size,
                              "device_attachment": device_attachment, "gpu_device": 0,
                              "gpu_process": True, "check_echo": True})
            before = s.gpu_calls
            p.run_requests(200)
            st = p.stats()
            assert st["success"] == 200 and st["error"] == 0, (size, st)
            assert s.gpu_calls - before == 200
    finally:
        s.stop()


@pytest.mark.parametrize("device_attachment", [False, True])
def test_gpu_process_echo_handler_bench_shape(dev, device_attachment):
    """The bench's GPU-handler leg shape: 50 in flight on one connection,
    64 KiB attachments, max_retry 0, every reply checked (bytes + device
    CRC). Any failure reports its error histogram."""
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    from brpc_amd.models.echo import ECHO_64KB
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    try:
        o = ECHO_64KB.press_options(s.address, gpu_device=0)
        o.update({"concurrency": 50, "check_echo": True, "check_every": 1, "gpu_process": True,
                  "device_attachment": device_attachment})
        p = native.Press(o)
        p.run_requests(2000)  # warm-up, as the bench does
        p.reset_stats()
        p.run_requests(20000)
        st = p.stats()
        assert st["success"] == 20000 and st["error"] == 0, (st["error_codes"], st["last_error"])
    finally:
        s.stop()


@pytest.mark.parametrize("mfma", [True, False])
def test_batched_copy_crc32c_fused(dev, mfma):
    """The fused pull+checksum kernels (CRC on the matrix cores, and on byte
    tables): bytes copied exactly, nothing written around the destination,
    and CRC32C equal to the host SSE4.2 value, aligned and misaligned
    segments alike."""
    from brpc_amd.ops import batched_copy_crc32c, crc32c_host
    big = torch.randint(0, 256, (1 << 21,), dtype=torch.uint8, device=dev)
    cases = [(0, 1), (3, 15), (0, 16), (5, 4099), (1, 65521), (16, 1 << 20), (7, (1 << 20) + 333), (0, 0),
             (9, 31), (2, 33), (0, 2048), (11, 4096 + 7), (0, 16384), (13, 16384 + 1), (0, 3 * 16384 - 5)]
    srcs = [big[o:o + n] for o, n in cases]
    outs = [torch.zeros(n + 32, dtype=torch.uint8, device=dev) for _, n in cases]
    dsts = [outs[i][3 + i % 8:3 + i % 8 + n] for i, (_, n) in enumerate(cases)]
    crcs = batched_copy_crc32c(srcs, dsts, mfma=mfma).cpu().tolist()
    torch.cuda.synchronize()
    for i, (s, d, c) in enumerate(zip(srcs, dsts, crcs)):
        assert torch.equal(s, d), i
        assert c == crc32c_host(s.cpu().numpy().tobytes()), i
        o = 3 + i % 8
        assert int(outs[i][:o].sum()) == 0 and int(outs[i][o + s.numel():].sum()) == 0, i


@pytest.mark.parametrize("mfma", ["true", "false"])
@pytest.mark.parametrize("size", [4096, 65536, 100003, 1 << 20])
def test_verified_device_pulls_over_rpc(dev, mfma, size):
    """-verify_device_payload on the RPC path with either CRC kernel: the
    sender's device CRC and the receiver's fused pull+CRC agree on every
    payload (no CRC failure), and the echoed bytes are right."""
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    native.set_flag("copy_engine_crc_mfma", mfma)
    native.set_flag("copy_engine_crc_mfma_min_bytes", "0")  # every launch takes the chosen kernel
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    try:
        before = native.gpu.xgmi_stats()["crc_failures"]
        p = native.Press({"server": s.address, "concurrency": 16, "attachment_size": size, "device_attachment": True,
                          "verify_device_payload": True, "gpu_device": 0, "check_echo": True, "check_every": 1,
                          "max_retry": 0})
        p.run_requests(400)
        st = p.stats()
        assert st["success"] == 400 and st["error"] == 0, (st["error_codes"], st["last_error"])
        assert native.gpu.xgmi_stats()["crc_failures"] == before
    finally:
        s.stop()
        native.set_flag("copy_engine_crc_mfma", "true")
        native.set_flag("copy_engine_crc_mfma_min_bytes", str(2 << 20))


@pytest.mark.parametrize("mfma", [True, False])
def test_copy_crc32c_checksum_only_segments(dev, mfma):
    """A null destination is a checksum-only segment (the verify path of
    payloads that stay where they are): the CRC is right and nothing is
    written."""
    from brpc_amd import native
    from brpc_amd.ops import crc32c_host
    from brpc_amd.ops._common import stream_handle
    sizes = [5, 4096, 16384 + 77, 1 << 20]
    srcs = [torch.randint(0, 256, (n + 3,), dtype=torch.uint8, device=dev)[3:] for n in sizes]
    out = torch.zeros(len(sizes), dtype=torch.int32, device=dev)
    native.gpu.batched_copy_crc32c_launch([s.data_ptr() for s in srcs], [0] * len(sizes), sizes, out.data_ptr(),
                                          stream_handle(dev), mfma)
    torch.cuda.synchronize()
    got = [(int(x) & 0xFFFFFFFF) for x in out.cpu().tolist()]
    assert got == [crc32c_host(s.cpu().numpy().tobytes()) for s in srcs]


def test_rpcz_annotates_device_pulls(dev, tmp_path):
    """rpcz: the xGMI pull done for a call is annotated in that call's span
    (server side: request attachment; client side: response attachment)
    and the spans land in the on-disk store, findable by trace id."""
    import re
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    native.set_flag("rpcz_database_dir", str(tmp_path))
    native.set_flag("enable_rpcz", "true")
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    try:
        p = native.Press({"server": s.address, "concurrency": 4, "attachment_size": 65536,
                          "device_attachment": True, "gpu_device": 0, "check_echo": True})
        p.run_requests(200)
        assert p.stats()["error"] == 0
        native.rpcz_flush()
        spans = native.rpcz_recent(400)
        gpu = [x for x in spans if "[gpu]" in x and "copy" in x]
        assert gpu, spans[:3]
        assert any(x.startswith("S ") for x in gpu), gpu[:3]
        assert any(x.startswith("C ") for x in gpu), gpu[:3]
        trace = int(re.search(r"trace=([0-9a-f]{16})", gpu[0]).group(1), 16)
        stored = native.rpcz_trace(trace)
        assert stored and any("[gpu]" in x for x in stored), stored
    finally:
        native.set_flag("enable_rpcz", "false")
        s.stop()


@pytest.mark.parametrize("mfma", [True, False])
def test_crc_kernels_need_no_zeroed_output(dev, mfma):
    """The copy+CRC kernel folds chunk CRCs through a per-stream scratch that
    every launch leaves zeroed, and STORES each result: garbage in the output
    buffer, repeated launches on one stream and multi-chunk segments give the
    same, correct CRCs (no memset launch per batch)."""
    from brpc_amd import native
    from brpc_amd.ops import crc32c_host
    from brpc_amd.ops._common import stream_handle
    sizes = [1, 16384, 16385, 65536, 200000, 1 << 20]
    srcs = [torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev) for n in sizes]
    dsts = [torch.empty(n, dtype=torch.uint8, device=dev) for n in sizes]
    want = [crc32c_host(s.cpu().numpy().tobytes()) for s in srcs]
    for rep in range(3):
        out = torch.full((len(sizes),), 0x5A5A5A5A, dtype=torch.int32, device=dev)
        native.gpu.batched_copy_crc32c_launch([s.data_ptr() for s in srcs], [d.data_ptr() for d in dsts], sizes,
                                              out.data_ptr(), stream_handle(dev), mfma)
        torch.cuda.synchronize()
        got = [(int(x) & 0xFFFFFFFF) for x in out.cpu().tolist()]
        assert got == want, rep
        for s, d in zip(srcs, dsts):
            assert torch.equal(s, d)


def test_fibers_park_on_long_kernels_while_rpcs_flow(dev):
    """SURVEY §7.1 / north star: tasks yield on hipEvent without blocking a
    pthread. 8 fibers wait on 100 ms kernels on a 2-worker runtime while 32 B
    echo calls keep completing on those same workers."""
    import json
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "gpu_park_probe.py")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    j = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert j["rcs"] == [0] * 8, j
    # every waiter really waited for its kernel...
    assert min(j["waited_us"]) >= 80000, j
    # ...and meanwhile the RPCs flowed on the 2 workers, none stalled
    assert j["errors"] == 0 and j["calls"] >= 500, j
    assert j["max_us"] < 50000, j


def test_dmabuf_export_of_real_hbm_registers_through_verbs(dev):
    """GPUDirect RDMA path with REAL HBM: an arena block is exported as a
    dmabuf fd by hipMemGetHandleForAddressRange (gpu/runtime.cc
    dmabuf_export_hook) and registered through the ibverbs provider's
    ibv_reg_dmabuf_mr — against the stub verbs library, since this pool has
    no HCA (the stub checks the fd and access flags, then records the
    registration)."""
    from brpc_amd import native
    lib = os.path.join(ROOT, "build", "lib", "libfake_ibverbs.so")
    d = native.gpu.dmabuf_register_probe(lib, 1 << 20, 0)
    assert d["arena_offset"] >= 0, d            # arena (IPC-exportable) memory
    assert d["export_rc"] == 0, d               # the real HIP export succeeded
    assert "dmabuf" in d["fd_target"], d        # and produced a dmabuf fd
    assert d["provider"] == "ibverbs", d
    assert d["register_rc"] == 0 and d["lkey"] != 0, d


_SPLIT_PROBE = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
from brpc_amd import native
from brpc_amd.models import start_echo_server
native.set_flag("hbm_arena_mb", "64")
s = start_echo_server("127.0.0.1:0", gpu_device=0)
def press(size, conc, n):
    p = native.Press({"server": s.address, "concurrency": conc, "attachment_size": size,
                      "device_attachment": True, "gpu_device": 0, "check_echo": True})
    p.run_requests(n)
    st = p.stats()
    assert st["success"] == n and st["error"] == 0, st
press(16 << 20, 2, 20)  # carves the whole 64 MiB arena in 16 MiB blocks (and then some)
a = native.gpu.hbm_pool_stats(0)
press(65536, 16, 2000)  # must be served by cutting up free 16 MiB blocks
b = native.gpu.hbm_pool_stats(0)
s.stop()
print(json.dumps({"a": a, "b": b}))
"""


def test_hbm_arena_splits_free_blocks_instead_of_falling_back(dev):
    """Once the arena is fully carved, a payload class with no free block
    is served by cutting up a free block of a larger class, not by a
    dedicated hipMalloc (slow, not lendable, synchronising hipFree)."""
    r = subprocess.run([sys.executable, "-c", _SPLIT_PROBE, ROOT], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    a, b = out["a"], out["b"]
    assert a["carved_bytes"] == 64 << 20, a
    assert b["splits"] > a["splits"], out
    assert b["fallback_allocs"] == a["fallback_allocs"], out
