"""RCCL data plane for RPC payloads (csrc/gpu/rccl_plane.h) on one MI355X.

A one-rank plane: client and server share the process and the GPU, so every
payload is a self send/receive pair issued in one RCCL group. The same code
path (sequence numbers in the meta, per-source ordering, drained rejects)
carries payloads between ranks on different GPUs; the multi-rank run is the
bench's rccl leg on an 8-GPU node (a one-GPU box cannot host two RCCL
ranks: profiles/r2_rccl_probe.txt)."""
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def plane():
    from brpc_amd import native, parallel
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    topo = parallel.Topology(rank=0, world_size=1, local_rank=0, local_world_size=1, device=0)
    native.set_flag("rccl_timeout_ms", "10000")
    assert parallel.init_rccl_plane(topo, min_bytes=65536)
    yield native
    parallel.set_rccl_min_bytes(None)


def _delta(a, b):
    return {k: b[k] - a[k] for k in a}


def test_echo_payloads_over_rccl(plane):
    native = plane
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    try:
        r0, x0 = native.gpu.rccl_stats(), native.gpu.xgmi_stats()
        p = native.Press({"server": s.address, "concurrency": 32, "attachment_size": 65536,
                          "device_attachment": True, "gpu_device": 0, "check_echo": True})
        p.run_requests(2000)
        st = p.stats()
        assert st["success"] == 2000 and st["error"] == 0, st
        r = _delta(r0, native.gpu.rccl_stats())
        x = _delta(x0, native.gpu.xgmi_stats())
        # request and response payloads (the first call of the connection is
        # staged while the hello is in flight)
        assert r["sent_payloads"] >= 3900 and r["recv_payloads"] >= 3900, r
        assert r["recv_bytes"] == r["recv_payloads"] * 65536, r
        assert r["aborts"] == 0 and r["discarded"] == 0, r
        # only the calls in flight before the connection's hello completed
        # (at most one per concurrent caller) were lent over xGMI
        assert x["copy_segments"] <= 64, x
        assert r["payload_rounds"] < r["sent_payloads"], r  # concurrent payloads share rounds
    finally:
        s.stop()


def test_small_payloads_stay_on_xgmi(plane):
    native = plane
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    try:
        r0, x0 = native.gpu.rccl_stats(), native.gpu.xgmi_stats()
        p = native.Press({"server": s.address, "concurrency": 8, "attachment_size": 16384,
                          "device_attachment": True, "gpu_device": 0, "check_echo": True})
        p.run_requests(500)
        st = p.stats()
        assert st["success"] == 500 and st["error"] == 0, st
        r = _delta(r0, native.gpu.rccl_stats())
        x = _delta(x0, native.gpu.xgmi_stats())
        assert r["sent_payloads"] == 0, r
        assert x["sent_payloads"] >= 900, x
    finally:
        s.stop()


def test_rejected_requests_drain_their_payloads(plane):
    """ELIMIT rejections never look at the attachment; the announced RCCL
    payload must still be received (into scratch) or the pair would stall."""
    native = plane
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0", gpu_device=0, max_concurrency=1)
    try:
        r0 = native.gpu.rccl_stats()
        p = native.Press({"server": s.address, "concurrency": 16, "attachment_size": 65536,
                          "device_attachment": True, "gpu_device": 0, "max_retry": 0})
        p.run_requests(1000)
        st = p.stats()
        assert st["error"] > 0 and st["success"] > 0, st
        r = _delta(r0, native.gpu.rccl_stats())
        assert r["discarded"] > 0 and r["aborts"] == 0, r
        # the plane is still in sync: a clean run afterwards
        s2 = start_echo_server("127.0.0.1:0", gpu_device=0)
        try:
            q = native.Press({"server": s2.address, "concurrency": 16, "attachment_size": 65536,
                              "device_attachment": True, "gpu_device": 0, "check_echo": True})
            q.run_requests(500)
            st2 = q.stats()
            assert st2["success"] == 500 and st2["error"] == 0, st2
        finally:
            s2.stop()
        assert native.gpu.rccl_stats()["aborts"] == 0
    finally:
        s.stop()


def test_stream_chunks_over_rccl(plane):
    native = plane
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0", gpu_device=0)
    try:
        r0 = native.gpu.rccl_stats()
        sp = native.StreamPress({"server": s.address, "chunk_size": 65536, "chunks_per_step": 32,
                                 "device_chunks": True, "gpu_device": 0})
        sp.run_steps(10)
        sp.close()
        r = _delta(r0, native.gpu.rccl_stats())
        assert r["recv_payloads"] >= 250 and r["aborts"] == 0, r
    finally:
        s.stop()
