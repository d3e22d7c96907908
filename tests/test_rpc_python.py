"""Python-facing RPC surface: Server/Channel/Press over loopback."""
import pytest
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_echo_roundtrip(native, echo_server):
    ch = native.Channel(echo_server.address)
    msg, att, lat = ch.echo("hello", b"\x00\x01payload")
    assert msg == "hello"
    assert att == b"\x00\x01payload"
    assert lat >= 0


def test_echo_large_attachment(native, echo_server):
    ch = native.Channel(echo_server.address)
    blob = bytes(range(256)) * 4096  # 1 MiB
    _, att, _ = ch.echo("big", blob)
    assert att == blob


def test_timeout_raises(native, echo_server):
    ch = native.Channel(echo_server.address, timeout_ms=50, max_retry=0)
    with pytest.raises(RuntimeError, match="E1008|timed out|Reached timeout"):
        ch.echo("slow", b"", sleep_us=300000)


def test_connection_refused(native):
    ch = native.Channel("127.0.0.1:1", timeout_ms=200, max_retry=0)
    with pytest.raises(RuntimeError):
        ch.echo("x")


def test_press_closed_loop(native, echo_server):
    p = native.Press({"server": echo_server.address, "concurrency": 16, "request_size": 32,
                      "check_echo": True})
    p.run_requests(5000)
    st = p.stats()
    assert st["success"] == 5000 and st["error"] == 0
    assert 0 < st["p50_us"] <= st["p99_us"] <= st["max_us"]
    assert st["qps"] > 1000


def test_press_attachment_checked(native, echo_server):
    p = native.Press({"server": echo_server.address, "concurrency": 4, "attachment_size": 65536,
                      "check_echo": True})
    p.run_requests(200)
    st = p.stats()
    assert st["success"] == 200, st


def test_press_open_loop_qps(native, echo_server):
    p = native.Press({"server": echo_server.address, "qps": 200.0, "concurrency": 2})
    p.run_for(1.0)
    st = p.stats()
    assert 120 <= st["success"] <= 260, st


def test_press_pooled_and_short(native, echo_server):
    for ct in ("pooled", "short"):
        p = native.Press({"server": echo_server.address, "concurrency": 8, "connection_type": ct})
        p.run_requests(400)
        assert p.stats()["success"] == 400


def test_press_generic_proto(native, echo_server, tmp_path):
    proto = tmp_path / "echo2.proto"
    proto.write_text('''
syntax = "proto2";
package example;
message EchoRequest { required string message = 1; optional int64 sleep_us = 2; }
message EchoResponse { required string message = 1; }
service EchoService { rpc Echo(EchoRequest) returns (EchoResponse); }
''')
    p = native.Press({"server": echo_server.address, "concurrency": 4, "proto_file": str(proto),
                      "method": "example.EchoService.Echo",
                      "input": '{"message": "a"} {"message": "bb"}'})
    p.run_requests(100)
    assert p.stats()["success"] == 100


def test_flags_and_vars(native, echo_server):
    from brpc_amd.utils import dump_vars, get_flag, list_flags, set_flag
    assert "fiber_concurrency" in list_flags()
    set_flag("log_unknown_protocol", True)
    assert get_flag("log_unknown_protocol") == "true"
    set_flag("log_unknown_protocol", False)
    v = dump_vars("*")
    assert len(v) > 10
    assert "rpc" in native.dump_prometheus() or len(native.dump_prometheus()) > 0


def test_press_over_rdma_soft_provider():
    """rdma_performance-style closed loop over the RDMA data plane (soft verbs
    provider: no HCA here). Runs in a child process because enabling RDMA swaps
    the process-wide Buf block allocator to the registered pool."""
    import subprocess
    import sys
    code = r'''
import json, sys
sys.path.insert(0, %r)
from brpc_amd import native
s = native.Server(); s.add_echo_service(); s.start("127.0.0.1:0", use_rdma=True)
out = {}
for att in (0, 1024, 65536, 1 << 20):
    p = native.Press({"server": s.address, "concurrency": 8, "attachment_size": att, "use_rdma": True,
                      "check_echo": True, "timeout_ms": 5000})
    p.run_requests(400 if att < (1 << 20) else 40)
    st = p.stats()
    out[att] = [st["success"], st["error"]]
s.stop()
print(json.dumps(out))
''' % (ROOT,)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    res = json.loads(r.stdout.strip().splitlines()[-1])
    for att, (ok, err) in res.items():
        assert err == 0, (att, res)
        assert ok == (400 if int(att) < (1 << 20) else 40), (att, res)


def test_stream_press_rounds_are_acknowledged(native, echo_server):
    sp = native.StreamPress({"server": echo_server.address, "chunk_size": 65536, "chunks_per_step": 8})
    sp.run_steps(5)
    st = sp.stats()
    assert st["steps"] == 5
    assert st["bytes_sent"] == st["bytes_acked"] == 5 * 8 * 65536
    sp.close()
