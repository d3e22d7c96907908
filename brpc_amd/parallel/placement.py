"""CPU placement of one rank: the L3 domain its fiber runtime is confined
to (-cpu_l3_domain, csrc/fiber/runtime.cc), chosen on the NUMA node its GPU
hangs off.

The MI355X boxes expose every CPU of the node to a container whose CPU-time
quota is a small fraction of them. Unconfined, the scheduler scatters the
runtime's threads over many L3 domains and both sockets; confined to one
L3 domain the 32 B echo is ~2x faster and stable. Pinned socket blocks and
the staging copies of a rank are DMA'd by its GPU, so the domain should sit
on that GPU's NUMA node (/sys/bus/pci/devices/<bdf>/local_cpulist); ranks
whose GPUs share a node take distinct domains of it.
"""
import os


def parse_cpulist(text):
    cpus = set()
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        else:
            cpus.add(int(part))
    return cpus


def allowed_cpus():
    try:
        return sorted(os.sched_getaffinity(0))
    except AttributeError:
        return list(range(os.cpu_count() or 1))


def l3_domains(cpus=None):
    """[(first_cpu, [cpus])] of the allowed CPUs grouped by shared L3, in the
    order the runtime's -cpu_l3_domain indexes them."""
    groups = {}
    for c in (cpus if cpus is not None else allowed_cpus()):
        first = c
        try:
            with open("/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list" % c) as f:
                first = int(f.read().split(",")[0].split("-")[0])
        except (OSError, ValueError):
            pass
        groups.setdefault(first, []).append(c)
    return sorted(groups.items())


def numa_nodes():
    """{node: set of CPUs} from /sys/devices/system/node, or {} when unreadable."""
    out = {}
    base = "/sys/devices/system/node"
    try:
        names = os.listdir(base)
    except OSError:
        return out
    for n in names:
        if n.startswith("node") and n[4:].isdigit():
            try:
                with open("%s/%s/cpulist" % (base, n)) as f:
                    out[int(n[4:])] = parse_cpulist(f.read())
            except OSError:
                pass
    return out


def gpu_numa(device, native=None):
    """(numa_node, set of local CPUs) of a GPU, or (-1, None) when unknown."""
    if device is None or device < 0:
        return -1, None
    try:
        if native is None:
            from .. import native as native_mod
            native = native_mod
        bdf = native.gpu.pci_bus_id(device)
    except Exception:  # noqa: BLE001 - no GPU runtime
        return -1, None
    if not bdf:
        return -1, None
    base = "/sys/bus/pci/devices/%s" % bdf
    node, cpus = -1, None
    try:
        with open(base + "/numa_node") as f:
            node = int(f.read().strip())
    except (OSError, ValueError):
        pass
    try:
        with open(base + "/local_cpulist") as f:
            cpus = parse_cpulist(f.read())
    except OSError:
        pass
    return node, cpus


def cpu_busy(seconds=0.2):
    """{cpu: busy fraction} over `seconds` from /proc/stat (every process on
    the host, not just ours), or {} when unreadable."""
    def snap():
        d = {}
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("cpu") and line[3].isdigit():
                    v = line.split()
                    t = list(map(int, v[1:]))
                    d[int(v[0][3:])] = (sum(t), t[3] + t[4])  # total, idle + iowait
        return d
    try:
        import time
        a = snap()
        time.sleep(seconds)
        b = snap()
    except (OSError, ValueError):
        return {}
    return {c: 1.0 - (b[c][1] - a[c][1]) / max(1, b[c][0] - a[c][0]) for c in a if c in b}


def host_cpus():
    """CPUs of the container's cpuset (what the domains are indexed over,
    also after the runtime confined this process to one of them)."""
    try:
        with open("/sys/fs/cgroup/cpuset.cpus.effective") as f:
            cpus = sorted(parse_cpulist(f.read()))
        if cpus:
            return cpus
    except OSError:
        pass
    return allowed_cpus()


def probe_domains(idxs, domains, seconds=0.5, native=None):
    """{domain index: {"late": wake-ups >150 us late, "run_delay_ms": ...,
    "nivcsw": ...}} from one pinned sleeper per CPU of every listed domain,
    all at once (fiber/cpu_probe.cc). {} without the native module."""
    if native is None:
        try:
            from .. import native as native_mod
            native = native_mod
        except Exception:  # noqa: BLE001
            return {}
    cpus = [c for i in idxs for c in domains[i][1]]
    try:
        res = native.probe_cpu_wake(cpus, int(seconds * 1000), 1000, 150)
    except Exception:  # noqa: BLE001
        return {}
    by_cpu = {r["cpu"]: r for r in res if r["wakes"] >= 0}
    out = {}
    for i in idxs:
        rs = [by_cpu[c] for c in domains[i][1] if c in by_cpu]
        if not rs:
            continue
        out[i] = {"late": sum(r["late_over"] for r in rs),
                  "run_delay_ms": round(sum(r["run_delay_us"] for r in rs) / 1000.0, 2),
                  "nivcsw": sum(r["nivcsw"] for r in rs),
                  "late_p99_us": max(r["late_p99_us"] for r in rs)}
    return out


def _quietest(mine, domains, sample_s, native, info):
    """Index of the domain in `mine` other tenants disturb least: fewest
    late wake-ups of pinned sleepers, then least runqueue delay; the busy
    share of /proc/stat when the probe is unavailable."""
    probe = probe_domains(mine, domains, sample_s, native)
    if probe:
        idx = min(probe, key=lambda i: (probe[i]["late"], probe[i]["nivcsw"], probe[i]["run_delay_ms"], i))
        info["l3_domain_probe"] = probe[idx]
        info["l3_domain_probe_worst_late"] = max(v["late"] for v in probe.values())
        return idx
    busy = cpu_busy(min(sample_s, 0.2))
    if not busy:
        return mine[0]
    load = {i: sum(busy.get(c, 0.0) for c in domains[i][1]) / len(domains[i][1]) for i in mine}
    idx = min(mine, key=lambda i: (round(load[i], 2), i))
    info["l3_domain_busy_pct"] = round(100.0 * load[idx], 1)
    info["l3_domain_busy_pct_max"] = round(100.0 * max(load.values()), 1)
    return idx


def choose_l3_domain(local_rank, local_world, device, device_count=0, native=None, sample_s=0.5,
                     widen_late=0):
    """Index (for -cpu_l3_domain) of the L3 domain this rank should use, and
    a description dict for the bench JSON. -1: leave the rank unconfined."""
    domains = l3_domains(host_cpus())
    info = {"l3_domains": len(domains)}
    if len(domains) <= 1:
        return -1, info
    node, local = gpu_numa(device, native)
    info["gpu_numa_node"] = node
    cand = list(range(len(domains)))
    if local:
        on_node = [i for i, (_, cs) in enumerate(domains) if set(cs) <= local]
        if on_node:
            cand = on_node
    # CPU 0's domain carries housekeeping and most IRQs
    if len(cand) > 1:
        cand = [i for i in cand if 0 not in domains[i][1]] or cand
    # spread the local ranks whose GPUs share this NUMA node over its domains
    peers = [local_rank]
    if device_count > 1 and node >= 0:
        peers = []
        for r in range(local_world):
            n, _ = gpu_numa(r % device_count, native)
            if n == node:
                peers.append(r)
        if local_rank not in peers:
            peers.append(local_rank)
    slot = sorted(peers).index(local_rank)
    # ranks sharing the node own disjoint slices of its domains; in its slice
    # a rank takes the domain the rest of the host disturbs least (other
    # jobs' threads preempting ours are what the tail latency is made of)
    mine = cand[slot::len(peers)] if len(cand) >= len(peers) else [cand[slot % len(cand)]]
    idx = mine[0]
    if len(mine) > 1 and sample_s > 0:
        idx = _quietest(mine, domains, sample_s, native, info)
    # a lone rank whose NUMA-local domains are all disturbed (the probe saw
    # more than widen_late late wake-ups in the best of them) may take a
    # quieter domain on another node: for small-message latency the host's
    # other tenants matter more than the GPU's PCIe locality
    probe = info.get("l3_domain_probe")
    if widen_late > 0 and local_world == 1 and probe and probe.get("late", 0) > widen_late and sample_s > 0:
        others = [i for i in range(len(domains)) if i not in mine and 0 not in domains[i][1]]
        if others:
            wide = {}
            idx2 = _quietest(others + [idx], domains, sample_s, native, wide)
            if idx2 != idx and wide.get("l3_domain_probe", {}).get("late", 1 << 30) < probe.get("late", 0):
                info["widened_from_probe"] = probe
                info["l3_domain_probe"] = wide["l3_domain_probe"]
                idx = idx2
                mine = mine + others
    info["l3_domain_candidates"] = len(mine)
    info["l3_domain_first_cpu"] = domains[idx][0]
    info["ranks_on_gpu_numa_node"] = len(peers)
    info["numa_local"] = bool(local) and set(domains[idx][1]) <= local
    return idx, info


def rechoose_l3_domain(local_rank, local_world, device, device_count=0, native=None, sample_s=0.5, widen_late=20):
    """Probe the rank's slice again and move the running process to its
    quietest domain (fiber::RebindL3Domain). Run right before a latency
    measurement: other tenants' load shifts over minutes. Returns the new
    placement dict ({} when nothing could be chosen)."""
    idx, info = choose_l3_domain(local_rank, local_world, device, device_count, native, sample_s, widen_late)
    if idx < 0:
        return {}
    if native is None:
        from .. import native as native_mod
        native = native_mod
    try:
        cur = int(native.get_flag("cpu_l3_domain"))
    except Exception:  # noqa: BLE001
        cur = -1
    info["l3_domain"] = idx
    info["moved"] = idx != cur
    if idx != cur and native.rebind_l3_domain(idx) != 0:
        info["moved"] = False
        info["error"] = "rebind failed"
    return info
