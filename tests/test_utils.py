"""brpc_amd.utils: typed flags, scoped overrides, --name=value lists,
Prometheus parsing and variable snapshots (CPU)."""
import pytest

from brpc_amd import native
from brpc_amd.models import start_echo_server
from brpc_amd.utils import (VarSnapshot, apply_flag_args, flag_overrides, get_flag, get_flag_typed,
                            parse_flag_args, parse_prometheus, set_flag, wait_for_var)


def test_typed_flags_and_overrides():
    before = get_flag("rccl_timeout_ms")
    with flag_overrides(rccl_timeout_ms=1234, event_dispatcher_spin_us=0):
        assert get_flag_typed("rccl_timeout_ms") == 1234
        assert isinstance(get_flag_typed("rccl_timeout_ms"), int)
    assert get_flag("rccl_timeout_ms") == before
    # a failing override restores what was already set
    with pytest.raises(ValueError):
        with flag_overrides(rccl_timeout_ms=99, no_such_flag_at_all=1):
            pass
    assert get_flag("rccl_timeout_ms") == before
    with pytest.raises(ValueError):
        set_flag("no_such_flag_at_all", 1)


def test_flag_argument_lists():
    assert parse_flag_args("--a=1 -b --c='x y'") == [("a", "1"), ("b", "true"), ("c", "x y")]
    assert parse_flag_args("") == []
    with pytest.raises(ValueError):
        parse_flag_args("a=1")
    before = get_flag("rccl_round_payloads")
    try:
        assert apply_flag_args("--rccl_round_payloads=77") == ["rccl_round_payloads"]
        assert get_flag_typed("rccl_round_payloads") == 77
    finally:
        set_flag("rccl_round_payloads", before)


def test_parse_prometheus():
    text = "\n".join([
        "# HELP rpc_count calls",
        "# TYPE rpc_count counter",
        "rpc_count 42",
        'rpc_latency{quantile="0.99",method="a\\"b"} 1.5e3',
        "process_uptime_s 7",
    ])
    m = parse_prometheus(text)
    assert m[("rpc_count", ())] == 42.0
    assert m[("rpc_latency", (("quantile", "0.99"), ("method", 'a"b')))] == 1500.0
    assert len(m) == 3
    with pytest.raises(ValueError):
        parse_prometheus("{bad} 1")


def test_snapshots_and_rates_follow_traffic():
    s = start_echo_server("127.0.0.1:0")
    try:
        ch = native.Channel(s.address)
        ch.echo("warm")
        a = VarSnapshot()
        for _ in range(20):
            ch.echo("x" * 32)
        b = VarSnapshot()
        d = b.delta(a)
        assert d, "no numeric variables"
        assert all(isinstance(v, float) for v in d.values())
        assert b.rates(a).keys() == d.keys()
        with pytest.raises(ValueError):
            a.rates(b)
        # every exposed variable renders as a valid Prometheus sample
        parsed = parse_prometheus(native.dump_prometheus())
        assert parsed
        name = next(iter(native.dump_vars("")))
        assert wait_for_var(name, lambda v: True, timeout=1) is not None
        with pytest.raises(TimeoutError):
            wait_for_var(name, lambda v: False, timeout=0.05)
    finally:
        s.stop()


def test_rccl_plane_api_on_cpu():
    """Without a GPU the plane is never joined; the threshold flag still
    round-trips (the bench toggles it around its rccl leg)."""
    from brpc_amd import parallel
    topo = parallel.Topology(rank=0, world_size=1, local_rank=0, local_world_size=1, device=-1)
    assert parallel.init_rccl_plane(topo) is False
    assert native.gpu.rccl_active() is False
    before = get_flag("rccl_min_bytes")
    try:
        parallel.set_rccl_min_bytes(32768)
        assert get_flag_typed("rccl_min_bytes") == 32768
        parallel.set_rccl_min_bytes(None)
        assert get_flag_typed("rccl_min_bytes") == 1 << 40
    finally:
        set_flag("rccl_min_bytes", before)
    st = parallel.rccl_stats()
    assert st["sent_payloads"] == 0 and st["aborts"] == 0
