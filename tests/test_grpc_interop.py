"""Wire compatibility with the reference gRPC implementation (grpcio):
grpcio client -> our h2/gRPC server, and our h2:grpc client -> grpcio
server. Messages are encoded by hand (protobuf wire format) so the test
needs no generated python stubs."""
from concurrent import futures

import pytest

grpc = pytest.importorskip("grpc")


def _varint(n):
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def _echo_req(msg):
    b = msg.encode()
    return b"\x0a" + _varint(len(b)) + b


def _parse_field1(data):
    assert data[0] == 0x0A
    n, i, shift = 0, 1, 0
    while True:
        b = data[i]
        n |= (b & 0x7F) << shift
        i += 1
        shift += 7
        if not b & 0x80:
            break
    return data[i:i + n].decode()


def test_grpcio_client_to_our_server(echo_server):
    with grpc.insecure_channel(echo_server.address) as ch:
        call = ch.unary_unary("/example.EchoService/Echo", request_serializer=lambda b: b,
                              response_deserializer=lambda b: b)
        for msg in ["hello", "x" * 70000, "ünïcødé"]:
            resp = call(_echo_req(msg), timeout=5)
            assert _parse_field1(resp) == msg
        # unknown method -> UNIMPLEMENTED
        bad = ch.unary_unary("/example.EchoService/Nope", request_serializer=lambda b: b,
                             response_deserializer=lambda b: b)
        with pytest.raises(grpc.RpcError) as ei:
            bad(_echo_req("x"), timeout=5)
        assert ei.value.code() == grpc.StatusCode.UNIMPLEMENTED


def test_our_client_to_grpcio_server(native):
    def handler(req, ctx):
        msg = _parse_field1(req)
        if msg == "fail":
            ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, "asked to fail")
        return _echo_req(msg[::-1])

    server = grpc.server(futures.ThreadPoolExecutor(max_workers=4))
    generic = grpc.method_handlers_generic_handler("example.EchoService", {
        "Echo": grpc.unary_unary_rpc_method_handler(handler, request_deserializer=lambda b: b,
                                                    response_serializer=lambda b: b)})
    server.add_generic_rpc_handlers((generic,))
    port = server.add_insecure_port("127.0.0.1:0")
    server.start()
    try:
        ch = native.Channel("127.0.0.1:%d" % port, protocol="h2:grpc", timeout_ms=5000)
        for msg in ["abc", "y" * 50000]:
            out, _, _ = ch.echo(msg)
            assert out == msg[::-1]
        with pytest.raises(RuntimeError, match="grpc-status 3"):
            ch.echo("fail")
    finally:
        server.stop(0)


@pytest.mark.parametrize("compression", ["Gzip", "Deflate"])
def test_grpcio_compressed_client_to_our_server(echo_server, compression):
    """grpc-encoding: the server decompresses the request through the
    compress registry and answers in the same encoding."""
    with grpc.insecure_channel(echo_server.address, compression=getattr(grpc.Compression, compression)) as ch:
        call = ch.unary_unary("/example.EchoService/Echo", request_serializer=lambda b: b,
                              response_deserializer=lambda b: b)
        for msg in ["small", "z" * 100000]:
            resp = call(_echo_req(msg), timeout=5)
            assert _parse_field1(resp) == msg


@pytest.mark.parametrize("ctype", [2, 3])  # gzip, zlib ("deflate")
def test_our_compressed_client_to_grpcio_server(native, ctype):
    seen = []

    def handler(req, ctx):
        seen.append(dict(ctx.invocation_metadata()).get("grpc-encoding"))
        return req  # echo as is

    server = grpc.server(futures.ThreadPoolExecutor(max_workers=4))
    generic = grpc.method_handlers_generic_handler("example.EchoService", {
        "Echo": grpc.unary_unary_rpc_method_handler(handler, request_deserializer=lambda b: b,
                                                    response_serializer=lambda b: b)})
    server.add_generic_rpc_handlers((generic,))
    port = server.add_insecure_port("127.0.0.1:0")
    server.start()
    try:
        p = native.Press({"server": "127.0.0.1:%d" % port, "protocol": "h2:grpc", "concurrency": 2,
                          "request_size": 20000, "request_compress_type": ctype, "check_echo": True,
                          "timeout_ms": 5000})
        p.run_requests(20)
        st = p.stats()
        assert st["success"] == 20 and st["error"] == 0, st
    finally:
        server.stop(0)


def test_snappy_grpc_between_our_ends(native, echo_server):
    """grpc-encoding: snappy (grpcio has no snappy; both ends are ours)."""
    p = native.Press({"server": echo_server.address, "protocol": "h2:grpc", "concurrency": 4,
                      "request_size": 70000, "request_compress_type": 1, "check_echo": True})
    p.run_requests(50)
    st = p.stats()
    assert st["success"] == 50 and st["error"] == 0, st


def test_compress_registry_roundtrip(native):
    import os
    data = os.urandom(5000) + b"abc" * 30000
    for t in (1, 2, 3):
        assert native.decompress(t, native.compress(t, data)) == data
    assert native.snappy_uncompress(native.compress(1, data)) == data
