"""CPU placement of a rank (brpc_amd/parallel/placement.py): L3 domain on
the GPU's NUMA node, disjoint between ranks sharing the node, and the least
busy one (host-wide /proc/stat load) within a rank's share."""
from brpc_amd.parallel import placement


def _fake_host(monkeypatch, busy):
    # 2 NUMA nodes x 4 L3 domains x 4 CPUs; GPUs 0-3 on node 0, 4-7 on node 1
    domains = [(d * 4, list(range(d * 4, d * 4 + 4))) for d in range(8)]
    monkeypatch.setattr(placement, "l3_domains", lambda cpus=None: domains)

    def gpu_numa(device, native=None):
        node = 0 if device % 8 < 4 else 1
        return node, set(range(node * 16, node * 16 + 16))

    monkeypatch.setattr(placement, "gpu_numa", gpu_numa)
    monkeypatch.setattr(placement, "cpu_busy", lambda seconds=0.2: busy)
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
