"""The RCCL payload plane (csrc/gpu/rccl_plane.h) across 2, 3 and 8 ranks on
the CPU: gloo for the control plane, the stub RCCL
(csrc/tests/stub/fake_rccl.cc) for the data plane — bounded shared-memory
FIFOs far smaller than a payload, and one in-order queue per process, so a
plane that could order a blocking send in front of the receive its peer
needs would hang here.

Every rank fans 64 KiB and 1 MiB attachments out to every other rank with 50
calls in flight (both directions of every pair at once) and checks every
echoed byte. Reference analog: the RDMA window/ACK-credit endpoint
(src/brpc/rdma/rdma_endpoint.cpp:771-895) and its rdma_performance harness.
"""
import json
import os
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(nranks, port, *extra, timeout=400):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
                            str(nranks), "--master-addr", "127.0.0.1", "--master-port", str(port),
                            os.path.join(ROOT, "tests", "plane_ranks.py"), "--out-dir", d] + list(extra),
                           capture_output=True, text=True, timeout=timeout, cwd="/tmp", env=env)
        assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
        outs = []
        for k in range(nranks):
            with open(os.path.join(d, "rank%d.json" % k)) as f:
                outs.append(json.load(f))
    return outs


def _check_legs(outs):
    n = len(outs)
    for o in outs:
        assert o["plane_up"] and o["host_memory"], o
        assert o["aborts"] == 0 and o["recv_timeouts"] == 0 and o["stash_expired"] == 0, o
        for leg in o["legs"]:
            assert leg["error"] == 0 and leg["success"] == leg["calls"], leg
    # every payload any rank sent was received by its peer (after the last
    # barrier every plane is quiet)
    assert sum(o["sent_payloads"] for o in outs) == sum(o["recv_payloads"] for o in outs)
    for k in range(len(outs[0]["legs"])):
        sent = sum(o["legs"][k]["sent_payloads"] for o in outs)
        calls = outs[0]["legs"][k]["calls"]
        # most calls' payloads (request and response to every peer) went
        # over the plane — only calls in flight before a connection's hello
        # came back used TCP
        assert sent >= n * (n - 1) * 2 * max(0, calls - 50) * 0.5, (k, sent)


@pytest.mark.parametrize("nranks", [2, 3])
def test_plane_fanout_both_directions(nranks):
    outs = _run(nranks, 29640 + nranks)
    _check_legs(outs)


def test_plane_eight_ranks_with_credit_stalls():
    # a 4 MiB window: 1 MiB payloads to 7 peers with 50 in flight must wait
    # for receiver credit, and still complete without deadlock
    outs = _run(8, 29650, "--window", str(4 << 20), "--calls", "200,16")
    _check_legs(outs)
    assert sum(leg["credit_stalls"] for o in outs for leg in o["legs"]) > 0


def test_plane_abort_propagates_to_every_rank():
    outs = _run(3, 29652, "--abort-test", "--sizes", "65536", "--calls", "100")
    for o in outs:
        # every rank saw rank 1's abort through the doorbell almost at once
        # (not after its own -rccl_timeout_ms watchdog)...
        assert not o["plane_active_after_abort"], o
        assert o["abort_noticed_ms"] < 1000, o
        # ...only calls in flight at that moment failed, and traffic went on
        # over the fallback
        assert o["abort_leg"]["success"] > 0 and o["abort_leg"]["error"] <= 3 * 50, o
        assert o["after_abort_leg"]["error"] == 0 and o["after_abort_leg"]["success"] == 100, o


def test_plane_refused_writes_leave_nothing_stashed():
    # with a 1-byte socket budget most requests are refused after their
    # payloads were queued on the plane: the controller cancels them, the
    # plane withdraws the unannounced ones and tells receivers to drop the
    # announced ones, so no receiver hoards payloads nobody will claim
    outs = _run(2, 29654, "--overcrowd-test", "--sizes", "65536", "--calls", "100")
    for o in outs:
        leg = o["overcrowd_leg"]
        assert leg["error"] > 0, leg
        assert leg["stash_payloads"] == 0 and leg["stash_bytes"] == 0, leg
        assert o["after_overcrowd_leg"] == {"success": 100, "error": 0}, o
        assert o["aborts"] == 0, o
    assert sum(o["overcrowd_leg"]["withdrawn"] for o in outs) > 0, [o["overcrowd_leg"] for o in outs]


def test_plane_slow_rank_stalls_only_its_own_pairs():
    # ring traffic (rank r calls only rank r+1) on 8 ranks; then rank 3's
    # poster sleeps 50 ms after every group. Only the pairs that include
    # rank 3 (2->3 and 3->4) may slow down: every other pair keeps its rate,
    # because a pair round fires only when both of its ranks are ready and a
    # group never waits behind another rank's work (round 3's node-wide
    # lockstep slowed every pair to the slow rank's pace).
    outs = _run(8, 29656, "--calls", "0,0", "--ring-test", "1.5", "--slow-rank", "3", "--slow-delay-us", "50000")
    slow_clients = {2, 3}
    for o in outs:
        assert o["aborts"] == 0 and o["recv_timeouts"] == 0, o
        full, slow = o["ring"]
        assert full["error"] == 0 and slow["error"] == 0, o
        assert full["qps"] > 0, o
    rates = {o["rank"]: (o["ring"][0]["qps"], o["ring"][1]["qps"]) for o in outs}
    # the slow rank's pairs: at most ~20 groups/s on its side
    for r in slow_clients:
        assert rates[r][1] < 0.5 * rates[r][0], rates
    # every other pair keeps at least half its full-speed rate (8 ranks share
    # this host's CPUs, so rates are noisy)
    for r, (full, slow) in rates.items():
        if r not in slow_clients:
            assert slow > 0.5 * full, (r, rates)


@pytest.mark.parametrize("pipeline", [0, 2])
def test_plane_one_rank_self_payloads(pipeline):
    """A one-rank plane: every payload goes from the rank to itself, moved
    by one batched copy per group (-rccl_self_copy), with up to
    -rccl_self_pipeline such groups in flight; every echoed byte checked."""
    outs = _run(1, 29760 + pipeline, "--calls", "300,30",
                "--flags", "rccl_self_pipeline=%d" % pipeline)
    _check_legs(outs)
    o = outs[0]
    for leg in o["legs"]:
        assert leg["sent_payloads"] >= leg["calls"], leg  # request and response both over the plane
        assert leg["sent_payloads"] == leg["recv_payloads"], leg
