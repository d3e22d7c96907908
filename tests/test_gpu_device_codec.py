"""Device-payload codec (gpu/device_codec.h): HBM attachments snappy-encoded
on the device, lent encoded, decoded by the receiver straight out of the lent
region, optionally pb_scan-indexed. Numerics against the host snappy codec
and the host protobuf serializer; RPC legs against the echoed bytes."""
import os
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    from brpc_amd import native
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    assert native.gpu.device_count() > 0, "native runtime sees no HIP device"
    return torch.device("cuda", 0)


def _varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _encode(native, data, dev):
    src = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    ulen, stride, nblocks = native.gpu.device_snappy_layout(len(data))
    region = torch.zeros(stride * nblocks, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()  # torch fills/copies run on its own stream
    clen = native.gpu.device_snappy_encode(src.data_ptr(), len(data), region.data_ptr(), 0)
    return region, ulen, stride, clen


@pytest.mark.parametrize("kind,size", [("text", 65536), ("text", 100003), ("random", 65536), ("const", 4096),
                                       ("text", 1), ("text", 1 << 20)])
def test_device_snappy_blocks_are_standard_snappy_and_round_trip(dev, kind, size):
    from brpc_amd import native
    data = native.echo_body(kind, size)
    region, ulen, stride, clen = _encode(native, data, dev)
    assert len(clen) == (size + ulen - 1) // ulen
    host = region.cpu().numpy().tobytes()
    # every block is a complete raw snappy stream the host codec decodes
    for i, c in enumerate(clen):
        assert 0 < c <= stride
        block = host[i * stride:i * stride + c]
        assert native.snappy_uncompress(block) == data[i * ulen:(i + 1) * ulen]
    # the device decoder rebuilds the payload from the table alone
    out = torch.zeros(size, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()  # torch fills/copies run on its own stream
    err, nf, _ = native.gpu.device_snappy_decode(region.data_ptr(), region.numel(), ulen, stride, clen,
                                                 out.data_ptr(), size, False, 0)
    assert err == 0
    assert out.cpu().numpy().tobytes() == data
    if kind == "text":
        assert sum(clen) < size * 0.6 or size < 4096


def test_device_snappy_decode_refuses_bad_tables(dev):
    from brpc_amd import native
    data = native.echo_body("text", 20000)
    region, ulen, stride, clen = _encode(native, data, dev)
    out = torch.zeros(len(data), dtype=torch.uint8, device=dev)
    before = native.gpu.device_codec_stats()["bad_tables"]
    bad = [
        (region.numel(), ulen, stride, clen[:-1]),                    # blocks do not cover the payload
        (region.numel(), ulen, stride, [stride + 1] + clen[1:]),       # block longer than its slot
        (stride * (len(clen) - 1), ulen, stride, clen),               # last block outside the region
        (region.numel(), ulen, stride, [1] + clen[1:]),               # a block without elements
        (region.numel(), 0, stride, clen),                            # no block size
    ]
    for rlen, u, st, cl in bad:
        torch.cuda.synchronize()  # torch fills/copies run on its own stream
        err, _, _ = native.gpu.device_snappy_decode(region.data_ptr(), rlen, u, st, cl, out.data_ptr(), len(data),
                                                    False, 0)
        assert err == 1, (rlen, u, st, cl[:3])
    assert native.gpu.device_codec_stats()["bad_tables"] - before == len(bad)
    # a corrupted block (valid table) is caught by the decoder, not trusted
    host = bytearray(region.cpu().numpy().tobytes())
    h = len(_varint(min(ulen, len(data))))
    for k in range(h, clen[0]):
        host[k] = 0xFF
    region2 = torch.frombuffer(host, dtype=torch.uint8).to(dev)
    torch.cuda.synchronize()  # torch fills/copies run on its own stream
    err, _, _ = native.gpu.device_snappy_decode(region2.data_ptr(), region2.numel(), ulen, stride, clen,
                                                out.data_ptr(), len(data), False, 0)
    assert err == 2


def test_device_snappy_decode_scans_the_message(dev):
    """pb_scan on the decoded bytes: the field table matches the host's
    serialization of the same message."""
    from brpc_amd import native
    body = native.echo_body("text", 50000)
    # EchoRequest{message = body (field 1, bytes), gpu_process = true (field 3)}
    msg = bytes([0x0A]) + _varint(len(body)) + body + bytes([0x18, 0x01])
    region, ulen, stride, clen = _encode(native, msg, dev)
    out = torch.zeros(len(msg), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()  # torch fills/copies run on its own stream
    err, nf, fields = native.gpu.device_snappy_decode(region.data_ptr(), region.numel(), ulen, stride, clen,
                                                      out.data_ptr(), len(msg), True, 0)
    assert err == 0 and nf == 2
    off = 1 + len(_varint(len(body)))
    assert fields[0] == (1 << 3) | 2 and fields[1] == (off << 32) | len(body)
    assert fields[2] == (3 << 3) | 0 and fields[3] == 1


def _echo(native, server, n, **extra):
    o = {"server": server, "concurrency": 16, "attachment_size": 65536, "device_attachment": True,
         "gpu_device": 0, "check_echo": True}
    o.update(extra)
    p = native.Press(o)
    p.run_requests(n)
    return p.stats()


@pytest.mark.parametrize("body", ["text", "const"])
def test_compressed_device_attachments_echo(dev, body):
    """Both directions encoded on the device (the server mirrors the
    client's choice), every echo checked byte for byte."""
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    try:
        x0, c0 = native.gpu.xgmi_stats(), native.gpu.device_codec_stats()
        st = _echo(native, s.address, 2000, attachment_body=body, device_compress=1)
        assert st["success"] == 2000 and st["error"] == 0, st
        x1, c1 = native.gpu.xgmi_stats(), native.gpu.device_codec_stats()
        # request and response of (almost) every call: the first calls of a
        # connection are staged over TCP while the hello is in flight
        assert x1["compressed_sent"] - x0["compressed_sent"] >= 3800, (x0, x1)
        assert x1["compressed_recv"] - x0["compressed_recv"] >= 3800, (x0, x1)
        assert c1["decodes"] - c0["decodes"] >= 3800, (c0, c1)
        assert c1["bad_tables"] == c0["bad_tables"] and c1["decode_errors"] == c0["decode_errors"]
        # what the lends carried: the encoded size, not the payload's
        assert c1["encoded_out_bytes"] - c0["encoded_out_bytes"] < 0.7 * (c1["encoded_bytes"] - c0["encoded_bytes"])
    finally:
        s.stop()


def test_incompressible_device_attachments_are_lent_raw(dev):
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    try:
        x0 = native.gpu.xgmi_stats()
        st = _echo(native, s.address, 500, attachment_body="random", device_compress=1)
        assert st["success"] == 500 and st["error"] == 0, st
        x1 = native.gpu.xgmi_stats()
        encoded_then_raw = x1["compress_skipped_raw"] - x0["compress_skipped_raw"]
        never_encoded = x1["compress_skipped_adaptive"] - x0["compress_skipped_adaptive"]
        # requests only: a request that arrived raw is echoed raw (the server
        # mirrors what it received). A few encodes while the in-flight calls
        # race the streak, then the adaptive skip (a probe every 32 payloads)
        # lends the rest raw without encoding
        assert encoded_then_raw + never_encoded >= 450, (x0, x1)
        assert never_encoded >= 300, (x0, x1)
        assert x1["compressed_sent"] == x0["compressed_sent"]
    finally:
        s.stop()


@pytest.mark.parametrize("compress", [0, 1])
def test_device_attachment_indexed_on_arrival(dev, compress):
    """The attachment is one serialized EchoRequest: the server gets its
    field table from the device, mirrors the scan, and the press checks the
    table of every reply."""
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    try:
        c0 = native.gpu.device_codec_stats()
        st = _echo(native, s.address, 1000, attachment_body="text", attachment_pb=True, device_scan=True,
                   device_compress=compress)
        assert st["success"] == 1000 and st["error"] == 0, st
        c1 = native.gpu.device_codec_stats()
        assert c1["scans"] - c0["scans"] >= 1900, (c0, c1)
    finally:
        s.stop()


def test_compressed_device_attachments_verified(dev):
    """CRC32C of the source on the sender, of the decoded bytes on the
    receiver (both on the device)."""
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    try:
        x0 = native.gpu.xgmi_stats()
        st = _echo(native, s.address, 1000, attachment_body="text", device_compress=1, verify_device_payload=True)
        assert st["success"] == 1000 and st["error"] == 0, st
        x1 = native.gpu.xgmi_stats()
        assert x1["crc_failures"] == x0["crc_failures"]
        assert x1["compressed_recv"] - x0["compressed_recv"] >= 1800
    finally:
        s.stop()


@pytest.mark.parametrize("compress", [0, 1])
def test_grpc_device_attachments_lent_encoded_and_indexed(dev, compress):
    """BASELINE config 4 on HBM bodies: the same device body over h2:grpc.
    The connection negotiates through the private SETTINGS parameter and the
    xGMI hello in mrpc-meta-bin; after that every request and response body
    is lent (device-snappy-encoded when asked), pb-scanned on arrival, and
    every reply checked byte for byte and against its field table."""
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    try:
        x0, c0 = native.gpu.xgmi_stats(), native.gpu.device_codec_stats()
        st = _echo(native, s.address, 1000, protocol="h2:grpc", attachment_body="text", attachment_pb=True,
                   device_scan=True, device_compress=compress)
        assert st["success"] == 1000 and st["error"] == 0, st
        x1, c1 = native.gpu.xgmi_stats(), native.gpu.device_codec_stats()
        # requests and responses, but for the first calls of the connection
        # (staged in-band while the hello is in flight)
        assert x1["recv_payloads"] - x0["recv_payloads"] >= 1900, (x0, x1)
        assert c1["scans"] - c0["scans"] >= 1900, (c0, c1)
        if compress:
            assert x1["compressed_recv"] - x0["compressed_recv"] >= 1900, (x0, x1)
            assert c1["decodes"] - c0["decodes"] >= 1900, (c0, c1)
        assert c1["bad_tables"] == c0["bad_tables"] and c1["decode_errors"] == c0["decode_errors"]
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


def test_compressed_device_attachments_cross_process(dev):
    """The receiver decodes out of ANOTHER process's arena (IPC-mapped)."""
    from brpc_amd import native
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    srv = subprocess.Popen([sys.executable, "-c", _SERVER_SCRIPT], stdin=subprocess.PIPE,
                           stdout=subprocess.PIPE, env=env, text=True)
    try:
        port = int(srv.stdout.readline())
        x0 = native.gpu.xgmi_stats()
        st = _echo(native, "127.0.0.1:%d" % port, 300, attachment_size=1 << 20, concurrency=4,
                   attachment_body="text", device_compress=1)
        assert st["success"] == 300 and st["error"] == 0, st
        x1 = native.gpu.xgmi_stats()
        assert x1["compressed_recv"] - x0["compressed_recv"] >= 250, (x0, x1)
    finally:
        srv.stdin.close()
        srv.wait(timeout=60)


# ---------------------------------------------------------------- packed runs
# kind -> (numpy dtype of the decoded array, wire value of each element)
_PB_KINDS = {
    0: ("int32", lambda a: a.astype("int64").view("uint64")),        # int32: sign-extended, 10 bytes if < 0
    1: ("uint32", lambda a: a.astype("uint64")),
    2: ("int32", lambda a: ((a.astype("int64") << 1) ^ (a.astype("int64") >> 63)).view("uint64") & 0xFFFFFFFF),
    3: ("int64", lambda a: a.view("uint64")),
    4: ("uint64", lambda a: a),
    5: ("int64", lambda a: ((a << 1) ^ (a >> 63)).view("uint64")),
    6: ("uint8", lambda a: a.astype("uint64")),
}


def _varints(np, wire):
    """Vectorized protobuf varint encoding of a uint64 array."""
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
    return out.tobytes()


def _values(np, kind, n, seed):
    rng = np.random.default_rng(seed)
    if kind == 6:
        return rng.integers(0, 2, n).astype(np.uint8)
    if kind in (0, 2):
        v = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
        v[::3] = rng.integers(-100, 100, len(v[::3]))  # short varints next to 5- and 10-byte ones
        return v
    if kind == 1:
        return rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) >> rng.integers(0, 32, n).astype(np.uint32)
    if kind in (3, 5):
        return rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64) >> rng.integers(0, 63, n)
    return rng.integers(0, 2**64 - 1, n, dtype=np.uint64) >> rng.integers(0, 64, n).astype(np.uint64)


@pytest.mark.parametrize("kind", sorted(_PB_KINDS))
def test_device_packed_runs_match_the_host(dev, kind):
    """Runs in HBM of 1, a few hundred and ~100k elements (one and many
    4 KiB chunks, varints straddling chunk edges) decoded in one request."""
    import numpy as np
    from brpc_amd import native
    dtype, wire_of = _PB_KINDS[kind]
    runs = [_values(np, kind, n, seed=kind * 10 + i) for i, n in enumerate((1, 333, 100003))]
    wires = [_varints(np, wire_of(v)) for v in runs]
    srcs = [torch.frombuffer(bytearray(w), dtype=torch.uint8).to(dev) for w in wires]
    esize = np.dtype(dtype).itemsize
    dsts = [torch.zeros(len(w) * esize, dtype=torch.uint8, device=dev) for w in wires]
    torch.cuda.synchronize()  # torch fills/copies run on its own stream
    res = native.gpu.device_decode_packed([s.data_ptr() for s in srcs], [len(w) for w in wires], [kind] * 3,
                                          [d.data_ptr() for d in dsts], 0)
    for v, w, d, (count, code) in zip(runs, wires, dsts, res):
        assert code == 0 and count == len(v), (len(w), count, code)
        got = np.frombuffer(d.cpu().numpy().tobytes()[:count * esize], dtype=dtype)
        want = v.astype(dtype) if kind != 6 else (v != 0).astype(np.uint8)
        assert np.array_equal(got, want)


def test_device_packed_runs_refuse_malformed_input(dev):
    from brpc_amd import native
    import numpy as np
    good = _varints(np, np.arange(1000, dtype=np.uint64) * 977)
    cases = [
        good[:-1] + bytes([good[-1] | 0x80]),    # ends inside a varint
        good + bytes([0xFF] * 10 + [0x01]),      # an 11-byte varint
        good[:5000] + bytes([0xFF] * 9 + [0x02]),  # a 10th byte above 1
    ]
    srcs = [torch.frombuffer(bytearray(c), dtype=torch.uint8).to(dev) for c in cases]
    dst = torch.zeros(8 * 20000, dtype=torch.uint8, device=dev)
    c0 = native.gpu.device_codec_stats()
    torch.cuda.synchronize()  # torch fills/copies run on its own stream
    res = native.gpu.device_decode_packed([s.data_ptr() for s in srcs] + [srcs[0].data_ptr()],
                                          [len(c) for c in cases] + [len(cases[0])], [4, 4, 4, 9],
                                          [dst.data_ptr()] * 4, 0)
    assert [code for _, code in res] == [1, 1, 1, 2], res
    assert native.gpu.device_codec_stats()["packed_errors"] - c0["packed_errors"] == 3


def test_packed_field_of_a_received_payload_stays_in_hbm(dev):
    """The whole HBM-resident path: a message with a packed int32 field and a
    bytes field is snappy-encoded on the device, decoded and scanned from the
    block table, and its packed field is located by the field table and
    decoded into a device array; no byte of it is read on the host."""
    import numpy as np
    from brpc_amd import native
    vals = _values(np, 0, 50000, seed=7)
    packed = _varints(np, _PB_KINDS[0][1](vals))
    blob = native.echo_body("text", 30000)
    msg = (bytes([0x0A]) + _varint(len(packed)) + packed + bytes([0x12]) + _varint(len(blob)) + blob)
    region, ulen, stride, clen = _encode(native, msg, dev)
    out = torch.zeros(len(msg), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()  # torch fills/copies run on its own stream
    err, nf, fields = native.gpu.device_snappy_decode(region.data_ptr(), region.numel(), ulen, stride, clen,
                                                      out.data_ptr(), len(msg), True, 0)
    assert err == 0 and nf == 2
    off, ln = native.gpu.device_payload_field(nf, fields, 1)
    assert ln == len(packed) and native.gpu.device_payload_field(nf, fields, 5) is None
    arr = torch.zeros(len(vals), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()  # torch fills/copies run on its own stream
    [(count, code)] = native.gpu.device_decode_packed([out.data_ptr() + off], [ln], [0], [arr.data_ptr()], 0)
    assert code == 0 and count == len(vals)
    assert np.array_equal(arr.cpu().numpy(), vals)


def test_codec_batch_limit_one_does_not_hold_a_requester(dev):
    """-codec_batch_max_inflight=1 under 50 calls in flight: every call
    finishes, and none waits for the whole burst. (A leader that launched
    batches while waiting on the oldest one kept its own finished RPC until
    the load stopped: a latency as long as the run.)"""
    import time
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    native.set_flag("codec_batch_max_inflight", "1")
    try:
        t0 = time.perf_counter()
        st = _echo(native, s.address, 6000, concurrency=50, attachment_body="text", device_compress=1)
        elapsed_us = (time.perf_counter() - t0) * 1e6
        assert st["success"] == 6000 and st["error"] == 0, st
        assert st["max_us"] < 0.5 * elapsed_us, (st["max_us"], elapsed_us)
    finally:
        native.set_flag("codec_batch_max_inflight", "6")
        s.stop()
