"""Fan-out workloads of the multi-GPU bench legs (BASELINE configs 2/3),
exercised on CPU: a ParallelChannel broadcast with attachment forwarding and
gathering, and one flow-controlled stream per peer server. On a GPU node the
same code moves HBM payloads over xGMI (tests/test_gpu_ops.py)."""
from brpc_amd.models import start_echo_server


def test_parallel_channel_fanout_with_attachments(native):
    servers = [start_echo_server("127.0.0.1:0") for _ in range(3)]
    try:
        p = native.Press({"server": servers[0].address,
                          "fanout_servers": ",".join(s.address for s in servers),
                          "concurrency": 8, "attachment_size": 4096, "check_echo": True})
        p.run_requests(300)
        st = p.stats()
        assert st["success"] == 300 and st["error"] == 0, st
        # every call reached every server
        assert [s.echo_calls for s in servers] == [300, 300, 300]
        # bytes = 2 directions x (message + attachment) x 3 peers
        assert st["bytes"] == 300 * 2 * (32 + 4096) * 3, st
    finally:
        for s in servers:
            s.stop()


def test_stream_press_fans_out_to_every_peer(native):
    servers = [start_echo_server("127.0.0.1:0") for _ in range(2)]
    try:
        sp = native.StreamPress({"server": ",".join(s.address for s in servers), "chunk_size": 65536,
                                 "chunks_per_step": 8})
        sp.run_steps(5)
        st = sp.stats()
        assert st["streams"] == 2 and st["steps"] == 5, st
        assert st["bytes_acked"] == 2 * 5 * 8 * 65536, st
        assert st["bytes_sent"] == st["bytes_acked"], st
        sp.close()
    finally:
        for s in servers:
            s.stop()


def test_gpu_process_without_gpu_fails_cleanly(native):
    s = start_echo_server("127.0.0.1:0")
    try:
        p = native.Press({"server": s.address, "concurrency": 2, "attachment_size": 100, "gpu_process": True,
                          "max_retry": 0})
        p.run_requests(4)
        st = p.stats()
        assert st["error"] == 4 and "GPU" in st["last_error"], st
    finally:
        s.stop()


def test_parallel_channel_scatter_gather(native):
    """TP analog: each server echoes its slice of the attachment; the
    gathered response is the original attachment (checked by the press)."""
    servers = [start_echo_server("127.0.0.1:0") for _ in range(3)]
    try:
        p = native.Press({"server": servers[0].address,
                          "fanout_servers": ",".join(s.address for s in servers), "scatter": True,
                          "concurrency": 8, "attachment_size": 65536, "check_echo": True})
        p.run_requests(200)
        st = p.stats()
        assert st["success"] == 200 and st["error"] == 0, st
        assert [s.echo_calls for s in servers] == [200, 200, 200]
        # bytes = 2 directions x (3 messages + one attachment in slices)
        assert st["bytes"] == 200 * 2 * (32 * 3 + 65536), st
    finally:
        for s in servers:
            s.stop()


def test_consistent_hash_routing_spreads_keys(native):
    """EP analog: every call carries a routing key; c_murmurhash sends each
    key to the server owning its shard, keys spread over all servers."""
    servers = [start_echo_server("127.0.0.1:0") for _ in range(4)]
    try:
        p = native.Press({"server": "list://" + ",".join(s.address for s in servers), "lb_policy": "c_murmurhash",
                          "concurrency": 4, "attachment_size": 1024, "check_echo": True})
        p.run_requests(800)
        st = p.stats()
        assert st["success"] == 800 and st["error"] == 0, st
        calls = [s.echo_calls for s in servers]
        assert sum(calls) == 800 and min(calls) > 800 // 16, calls
    finally:
        for s in servers:
            s.stop()


def test_stream_relay_chain(native):
    """PP analog: chunks pushed into server A are relayed A -> B -> C in
    order; C's acknowledgements travel back, so steps complete end to end."""
    servers = [start_echo_server("127.0.0.1:0") for _ in range(3)]
    try:
        sp = native.StreamPress({"server": servers[0].address, "chunk_size": 65536, "chunks_per_step": 8,
                                 "relay_chain": ",".join(s.address for s in servers[1:])})
        sp.run_steps(6)
        st = sp.stats()
        assert st["streams"] == 1 and st["steps"] == 6, st
        assert st["bytes_acked"] == 6 * 8 * 65536, st
        sp.close()
        # every hop saw the set-up call: A (from the press), B (from A), C (from B)
        assert [s.echo_calls for s in servers] == [1, 1, 1]
    finally:
        for s in servers:
            s.stop()


def test_stream_relay_to_unreachable_hop_fails(native):
    import pytest
    s = start_echo_server("127.0.0.1:0")
    try:
        with pytest.raises(Exception):
            native.StreamPress({"server": s.address, "chunk_size": 4096, "chunks_per_step": 2,
                                "relay_chain": "127.0.0.1:1"})
    finally:
        s.stop()
