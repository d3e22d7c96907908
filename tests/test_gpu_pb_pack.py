"""Device body encode and JSON number arrays (K6):
pb_run_encode_kernel against the python protobuf varint / JSON rules for
every element kind and both formats, chunk boundaries, and the RPC path
where the GPU snappy codec leaves large packed fields of the body to the
kernel (baidu_std and gRPC, every echoed id checked)."""
import json
import random
import struct

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

KINDS = {"int32": (0, "i"), "uint32": (1, "I"), "sint32": (2, "i"), "int64": (3, "q"), "uint64": (4, "Q"),
         "sint64": (5, "q"), "bool": (6, "B")}


def _varint(v):
    v &= (1 << 64) - 1
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _ref(kind, vals, fmt):
    if fmt == 1:
        if kind == "bool":
            return ",".join("true" if v else "false" for v in vals).encode()
        return ",".join(str(v) for v in vals).encode()
    out = bytearray()
    for v in vals:
        if kind == "sint32":
            v = ((v << 1) ^ (v >> 31)) & 0xFFFFFFFF
        elif kind == "sint64":
            v = ((v << 1) ^ (v >> 63)) & ((1 << 64) - 1)
        elif kind == "bool":
            v = 1 if v else 0
        out += _varint(v)
    return bytes(out)


def _values(kind, n, seed):
    rnd = random.Random(seed)
    bits = {"int32": 32, "uint32": 32, "sint32": 32, "int64": 64, "uint64": 64, "sint64": 64, "bool": 1}[kind]
    signed = kind in ("int32", "sint32", "int64", "sint64")
    edge = [0, 1, 127, 128, 16383, 16384]
    if signed:
        edge += [-1, -(1 << (bits - 1)), (1 << (bits - 1)) - 1]
    elif bits > 1:
        edge += [(1 << bits) - 1]
    vals = []
    for i in range(n):
        if kind == "bool":
            vals.append(rnd.getrandbits(1))
        elif i < len(edge):
            vals.append(edge[i])
        else:
            w = rnd.randint(1, bits)
            v = rnd.getrandbits(w)
            if signed:
                v = v - (1 << (w - 1)) if w > 1 else -v
                v = max(-(1 << (bits - 1)), min((1 << (bits - 1)) - 1, v))
            vals.append(v)
    return vals


@pytest.fixture(scope="module")
def native():
    from brpc_amd import native as n
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    n.gpu.init(0)
    return n


@pytest.mark.parametrize("kind", sorted(KINDS))
@pytest.mark.parametrize("fmt", [0, 1])
@pytest.mark.parametrize("n", [1, 255, 256, 2047, 2048, 2049, 10000])
def test_run_encode_matches_reference(native, kind, fmt, n):
    code, pk = KINDS[kind]
    vals = _values(kind, n, seed=n * 31 + code * 7 + fmt)
    raw = struct.pack("<%d%s" % (n, pk), *vals)
    got = native.gpu.pb_run_encode(raw, n, code, fmt, 0)
    assert got == _ref(kind, vals, fmt)
    if fmt == 1:
        # a JSON array of the same numbers
        parsed = json.loads(b"[" + got + b"]")
        assert parsed == ([bool(v) for v in vals] if kind == "bool" else vals)


@pytest.mark.parametrize("kind", sorted(KINDS))
@pytest.mark.parametrize("n", [1, 100, 4095, 4096, 5000, 40000])
def test_run_decode_matches_reference(native, kind, n):
    """Varint payload -> vector layout on the device (pb_run_count/decode
    kernels): varints straddling the 4 KiB chunk edges, every length."""
    code, pk = KINDS[kind]
    vals = _values(kind, n, seed=n * 17 + code)
    payload = _ref(kind, vals, 0)
    got = native.gpu.pb_run_decode(payload, code, 0)
    want = struct.pack("<%d%s" % (n, pk), *[(1 if v else 0) if kind == "bool" else v for v in vals])
    assert got == want


def test_run_decode_round_trips_the_encoder(native):
    vals = _values("sint64", 20000, seed=5)
    raw = struct.pack("<20000q", *vals)
    enc = native.gpu.pb_run_encode(raw, 20000, 5, 0, 0)
    assert native.gpu.pb_run_decode(enc, 5, 0) == raw


def test_run_decode_rejects_malformed(native):
    with pytest.raises(RuntimeError):
        native.gpu.pb_run_decode(b"\x01\x80", 3, 0)  # truncated: ends on a continuation byte
    with pytest.raises(RuntimeError):
        native.gpu.pb_run_decode(b"\x01" + b"\xff" * 10 + b"\x01", 3, 0)  # 11-byte varint
    with pytest.raises(RuntimeError):
        native.gpu.pb_run_decode(b"\xff" * 9 + b"\x02", 4, 0)  # 10th byte above 1
    # 10 bytes with a final 0x01 is 2**63 and fine
    assert native.gpu.pb_run_decode(b"\x80" * 9 + b"\x01", 4, 0) == struct.pack("<Q", 1 << 63)


def test_run_encode_rejects_bad_kind(native):
    with pytest.raises(RuntimeError):
        native.gpu.pb_run_encode(b"\0" * 8, 1, 99, 0, 0)


@pytest.mark.parametrize("protocol", ["baidu_std", "h2:grpc"])
def test_packed_ids_encoded_on_device_in_the_codec_batch(native, protocol):
    """Requests and responses carrying 16k packed int64 ids with snappy on
    the GPU codec: the serializer leaves the ids to pb_run_encode_kernel
    (pack_runs counts them), the body is compressed after it in the same
    batch, and the server/client parse every id back exactly."""
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    native.gpu.enable_snappy(0, 16384)
    try:
        b0 = native.gpu.snappy_stats()
        c0 = native.gpu.codec_batch_stats()
        p = native.Press({"server": s.address, "protocol": protocol, "concurrency": 16, "request_size": 16,
                          "packed_ids": 16384, "request_compress_type": 1, "check_echo": True})
        p.run_requests(200)
        st = p.stats()
        assert st["success"] == 200 and st["error"] == 0, st
        b1 = native.gpu.snappy_stats()
        c1 = native.gpu.codec_batch_stats()
        # one run of 8 chunks per request on the client; gRPC answers with
        # the request's grpc-encoding, so its responses are packed on the
        # server too (a baidu_std server compresses only when its handler
        # sets a response compress type, as in the reference)
        bodies = 400 if protocol == "h2:grpc" else 200
        assert b1["pack_runs"] - b0["pack_runs"] >= bodies, (b0, b1)
        assert b1["pack_run_chunks"] - b0["pack_run_chunks"] >= bodies * 8, (b0, b1)
        assert c1["run_chunks"] - c0["run_chunks"] >= bodies * 8, (c0, c1)
        # the receiving side decodes the ids on the device too (request on
        # the server always; gRPC responses on the client)
        assert b1["unpack_runs"] - b0["unpack_runs"] >= bodies, (b0, b1)
        assert c1["decode_chunks"] - c0["decode_chunks"] > 0, (c0, c1)
        assert b1["fallbacks"] == b0["fallbacks"], (b0, b1)
    finally:
        native.gpu.disable_snappy()
        s.stop()


def test_plain_bodies_go_to_the_cpu_codec_by_default(native):
    """-gpu_snappy_packed_only (the default of enable_snappy): 64 KiB text
    bodies without packed ids are compressed by the CPU codec on the send
    side (plain_routed counts them) and, after one probing device decode
    per type and worker, decoded by the CPU codec too."""
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    native.gpu.enable_snappy(0, 16384)
    try:
        b0 = native.gpu.snappy_stats()
        p = native.Press({"server": s.address, "protocol": "baidu_std", "concurrency": 8, "request_size": 65536,
                          "body": "text", "request_compress_type": 1, "check_echo": True})
        p.run_requests(400)
        st = p.stats()
        assert st["success"] == 400 and st["error"] == 0, st
        b1 = native.gpu.snappy_stats()
        assert b1["pack_runs"] == b0["pack_runs"]
        assert b1["compress_calls"] == b0["compress_calls"], (b0, b1)
        assert b1["plain_routed"] - b0["plain_routed"] >= 400, (b0, b1)
        # device decodes only as probes: at most one per 32 bodies per worker
        # (requests on the server, responses on the client; a worker probes each type once before it skips)
        assert b1["indexed_parses"] - b0["indexed_parses"] <= 2 * (400 // 32) + 32, (b0, b1)
    finally:
        native.gpu.disable_snappy()
        s.stop()


def test_packed_ids_below_threshold_stay_on_host(native):
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    native.gpu.enable_snappy(0, 16384)
    try:
        b0 = native.gpu.snappy_stats()
        p = native.Press({"server": s.address, "protocol": "baidu_std", "concurrency": 4, "request_size": 20000,
                          "packed_ids": 1000, "request_compress_type": 1, "check_echo": True})
        p.run_requests(50)
        assert p.stats()["success"] == 50
        assert native.gpu.snappy_stats()["pack_runs"] == b0["pack_runs"]
    finally:
        native.gpu.disable_snappy()
        s.stop()


def test_http_json_ids_printed_on_device(native):
    """http + json echo of 16k ids: with the GPU JSON path on, pb2json of
    both the request (client) and the response (server) hands the id array
    to the device printer, and every id parses back exactly."""
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    native.gpu.enable_json_index(0, 16384)
    try:
        j0 = native.gpu.json_stats()
        p = native.Press({"server": s.address, "protocol": "http", "connection_type": "pooled", "concurrency": 8,
                          "request_size": 16, "packed_ids": 16384, "check_echo": True})
        p.run_requests(100)
        st = p.stats()
        assert st["success"] == 100 and st["error"] == 0, st
        j1 = native.gpu.json_stats()
        assert j1["pb2json_arrays"] - j0["pb2json_arrays"] >= 200, (j0, j1)
        assert j1["pb2json_elems"] - j0["pb2json_elems"] >= 200 * 16384, (j0, j1)
        assert j1["pb2json_failures"] == j0["pb2json_failures"]
        # and the receiving json2pb parses the id arrays on the device
        assert j1["int_arrays"] - j0["int_arrays"] >= 200, (j0, j1)
    finally:
        native.gpu.disable_json_index()
        s.stop()


def test_json_int_arrays_parsed_on_device(native):
    """json2pb of an indexed body: a plain integer array (int64 extremes,
    whitespace, negative zero) is parsed by json_int_array_kernel; an array
    holding a float falls back to the element-wise parser, which reports
    the bad element exactly as before."""
    ids = [0, -1, 1, (1 << 63) - 1, -(1 << 63)] + [((i * 7919) << (i % 37)) * (-1 if i % 3 == 0 else 1)
                                                 for i in range(6000)]
    body = '{"message":"m","ids":[' + ", ".join(str(x) for x in ids[:10]) + "," + \
        ",".join(str(x) for x in ids[10:]) + ", -0 ]}"
    native.gpu.enable_json_index(0, 1024)
    try:
        j0 = native.gpu.json_stats()
        out = native.json_to_pb_to_json("example.EchoRequest", body.encode())
        j1 = native.gpu.json_stats()
        assert j1["int_arrays"] - j0["int_arrays"] == 1, (j0, j1)
        assert json.loads(out)["ids"] == ids + [0]
        bad = body.replace('"ids":[', '"ids":[1.5,', 1)
        with pytest.raises(RuntimeError):
            native.json_to_pb_to_json("example.EchoRequest", bad.encode())
        j2 = native.gpu.json_stats()
        assert j2["int_array_fallbacks"] - j1["int_array_fallbacks"] == 1, (j1, j2)
    finally:
        native.gpu.disable_json_index()
