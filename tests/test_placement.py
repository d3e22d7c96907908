"""CPU placement of a rank (brpc_amd/parallel/placement.py): L3 domain on
the GPU's NUMA node, disjoint between ranks sharing the node, and within a
rank's share the one other tenants disturb least (pinned-sleeper wake-up
probe, fiber/cpu_probe.cc; host-wide /proc/stat load without it)."""
import os
import subprocess
import sys

from brpc_amd.parallel import placement


def _fake_host(monkeypatch, busy, probe=None):
    # 2 NUMA nodes x 4 L3 domains x 4 CPUs; GPUs 0-3 on node 0, 4-7 on node 1
    domains = [(d * 4, list(range(d * 4, d * 4 + 4))) for d in range(8)]
    monkeypatch.setattr(placement, "l3_domains", lambda cpus=None: domains)

    def gpu_numa(device, native=None):
        node = 0 if device % 8 < 4 else 1
        return node, set(range(node * 16, node * 16 + 16))

    monkeypatch.setattr(placement, "gpu_numa", gpu_numa)
    monkeypatch.setattr(placement, "cpu_busy", lambda seconds=0.2: busy)
    monkeypatch.setattr(placement, "host_cpus", lambda: list(range(32)))
    if probe is None:
        monkeypatch.setattr(placement, "probe_domains", lambda idxs, domains, seconds=0.5, native=None: {})
    else:
        monkeypatch.setattr(placement, "probe_domains",
                            lambda idxs, domains, seconds=0.5, native=None: {i: probe[i] for i in idxs if i in probe})
    return domains


def test_single_rank_takes_least_busy_domain_of_its_node(monkeypatch):
    busy = {c: 0.5 for c in range(32)}
    for c in range(8, 12):  # domain 2 idle
        busy[c] = 0.0
    _fake_host(monkeypatch, busy)
    idx, info = placement.choose_l3_domain(0, 1, 0, device_count=8)
    assert idx == 2 and info["numa_local"] and info["l3_domain_busy_pct"] == 0.0


def test_domain_of_cpu0_is_avoided(monkeypatch):
    busy = {c: 0.5 for c in range(32)}
    for c in range(0, 4):  # CPU 0's domain idle but reserved for housekeeping
        busy[c] = 0.0
    _fake_host(monkeypatch, busy)
    idx, _ = placement.choose_l3_domain(0, 1, 0, device_count=8)
    assert idx != 0


def test_ranks_sharing_a_node_get_disjoint_domains(monkeypatch):
    _fake_host(monkeypatch, {c: 0.0 for c in range(32)})
    picks = [placement.choose_l3_domain(r, 8, r, device_count=8)[0] for r in range(8)]
    assert len(set(picks[:4])) == 3  # node 0 has 3 usable domains (CPU 0's is skipped) for 4 ranks
    assert all(p < 4 for p in picks[:4]) and all(p >= 4 for p in picks[4:])
    assert len(set(picks[4:])) == 4


def test_cpu_busy_reads_proc_stat():
    b = placement.cpu_busy(0.05)
    assert b and all(0.0 <= v <= 1.0 for v in b.values())


def test_probe_picks_the_domain_with_fewest_late_wakeups(monkeypatch):
    def row(late, nivcsw=0):
        return {"late": late, "run_delay_ms": 1.0, "nivcsw": nivcsw, "late_p99_us": 10}
    probe = {1: row(40), 2: row(3, 5), 3: row(3, 1)}
    _fake_host(monkeypatch, {c: 0.0 for c in range(32)}, probe)
    idx, info = placement.choose_l3_domain(0, 1, 0, device_count=8)
    assert idx == 3 and info["l3_domain_probe"]["late"] == 3 and info["l3_domain_probe_worst_late"] == 40


def test_native_wake_probe_measures_allowed_cpus():
    from brpc_amd import native
    cpus = sorted(os.sched_getaffinity(0))[:2]
    res = native.probe_cpu_wake(cpus + [100000], 100, 1000, 150)
    assert [r["cpu"] for r in res] == cpus + [100000]
    for r in res[:2]:
        assert 30 <= r["wakes"] <= 101 and r["late_p50_us"] <= r["late_p99_us"] <= r["late_max_us"]
        assert r["run_delay_us"] >= 0 and r["nivcsw"] >= 0
    assert res[2]["wakes"] == -1  # not a CPU we may run on


def test_rebind_moves_every_thread():
    code = r"""
import os, sys, threading, time
sys.path.insert(0, sys.argv[1])
from brpc_amd import native
from brpc_amd.parallel import placement
native.set_flag("cpu_l3_domain", "0")
native.set_concurrency(2)
native.Press  # runtime up through the module
doms = placement.l3_domains(placement.host_cpus())
k = len(doms) - 1
assert native.rebind_l3_domain(k) == 0
want = set(doms[k][1])
for tid in os.listdir("/proc/self/task"):
    assert os.sched_getaffinity(int(tid)) == want, tid
assert native.get_flag("cpu_l3_domain") == str(k)
print("ok", k)
"""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code, root], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def test_hw_queues_per_rank_keeps_shared_gpus_within_the_queue_budget(monkeypatch):
    """Ranks sharing a GPU split its mapped compute queues (num_cp_queues):
    8 ranks on one 24-queue GPU get 2 each (+1 of HIP's own = 24); one rank
    per GPU keeps HIP's default of 4."""
    from brpc_amd.parallel import topology
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("CUDA_VISIBLE_DEVICES", raising=False)
    monkeypatch.setattr(topology, "_kfd_gpu_nodes", lambda: [24])
    assert topology.hw_queues_per_rank(1) == 4
    assert topology.hw_queues_per_rank(2) == 4
    assert topology.hw_queues_per_rank(4) == 4
    assert topology.hw_queues_per_rank(8) == 2
    assert topology.hw_queues_per_rank(16) == 1
    monkeypatch.setattr(topology, "_kfd_gpu_nodes", lambda: [24] * 8)
    assert topology.hw_queues_per_rank(8) == 4  # one rank per GPU
    monkeypatch.setattr(topology, "_kfd_gpu_nodes", lambda: [])
    assert topology.hw_queues_per_rank(8) == 4  # no KFD (CPU host): HIP's default
