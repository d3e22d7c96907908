"""Rank topology for one-process-per-GPU jobs.

torchrun exports RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT. The
torch process group is only the job's CONTROL plane — address exchange,
the RCCL plane's unique id, barriers and result reductions — and it runs on
gloo by default, GPU or not. The RPC data moves over the framework's own
transports: TCP, xGMI lending, and the RCCL payload plane
(csrc/gpu/rccl_plane.h), which owns its own communicator and stream.

Why not torch's "nccl" backend for the barriers: its collectives are RCCL
kernels on torch's streams. With GPU_MAX_HW_QUEUES=4 those streams share
hardware queues with the payload plane's stream, and two blocking RCCL
kernels queued in opposite orders on two ranks (a barrier behind a plane
round on one, a plane round behind the barrier on the other) would wait
for each other forever. Set MRPC_DIST_BACKEND=nccl to use it anyway.
"""
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class Topology:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    local_world_size: int = 1
    device: int = -1          # GPU ordinal, -1 on CPU-only hosts
    backend: str = ""

    @property
    def distributed(self):
        return self.world_size > 1


def init_distributed(prefer_gpu=True):
    """Initialise from torchrun's env; a no-op single-rank topology when
    WORLD_SIZE is unset or 1."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    lrank = int(os.environ.get("LOCAL_RANK", str(rank)))
    lws = int(os.environ.get("LOCAL_WORLD_SIZE", str(ws)))
    use_gpu = prefer_gpu and torch.cuda.is_available()
    device = -1
    if use_gpu:
        device = lrank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(device)
    backend = ""
    if ws > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("MRPC_DIST_BACKEND", "gloo") if use_gpu else "gloo"
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", device)
        dist.init_process_group(backend=backend, rank=rank, world_size=ws, **kw)
    elif dist.is_initialized():
        backend = dist.get_backend()
    return Topology(rank, ws, lrank, lws, device, backend)


def _kfd_gpu_nodes():
    """num_cp_queues of every GPU this process can open, from the KFD
    topology in sysfs: no HIP call, so it can run before the runtime starts.
    A container sees every GPU of the host in the topology but can open only
    its own render nodes (/dev/dri/renderD<drm_render_minor>)."""
    import glob
    out = []
    for path in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties")):
        props = {}
        try:
            with open(path) as f:
                for line in f:
                    k, _, v = line.strip().partition(" ")
                    props[k] = v
        except OSError:
            continue
        if int(props.get("simd_count", "0") or 0) <= 0:
            continue
        minor = props.get("drm_render_minor")
        if minor is not None and not os.access("/dev/dri/renderD%s" % minor, os.R_OK | os.W_OK):
            continue
        out.append(int(props.get("num_cp_queues", "0") or 0))
    return out


def hw_queues_per_rank(local_world_size, default=4):
    """Hardware queues each rank's HIP runtime may create (GPU_MAX_HW_QUEUES)
    when several ranks share a GPU. The GPU maps at most num_cp_queues
    compute queues of all its processes at once (24 on the MI355X boxes,
    KFD topology); beyond that the scheduler time-slices the queues, and a
    kernel waits hundreds of microseconds for its queue's turn. Measured, 8
    ranks on one GPU (4 streams + 1 internal queue each = 40 queues):
    echo_64KB 18k QPS; with 2 queues each: 569k (profiles/r6_xproc_diagnosis.txt).
    One rank per GPU keeps the default."""
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
    nodes = _kfd_gpu_nodes()
    ngpu = len([x for x in vis.split(",") if x.strip()]) if vis else len(nodes)
    if ngpu <= 0 or local_world_size <= ngpu:
        return default
    per_gpu = (local_world_size + ngpu - 1) // ngpu
    cp = min(nodes) if nodes and min(nodes) > 0 else 24
    # one queue per rank is HIP's own (null stream / internal copies)
    return max(1, min(default, cp // per_gpu - 1))


def _tensor(x, topo):
    dev = torch.device("cuda", topo.device) if topo.backend == "nccl" else torch.device("cpu")
    return torch.tensor([x], dtype=torch.float64, device=dev)


def barrier(topo):
    if topo.distributed:
        if topo.backend == "nccl":
            dist.barrier(device_ids=[topo.device])
        else:
            dist.barrier()


def allreduce_max(x, topo):
    if not topo.distributed:
        return float(x)
    t = _tensor(x, topo)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allreduce_sum(x, topo):
    if not topo.distributed:
        return float(x)
    t = _tensor(x, topo)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def exchange_addresses(addr, topo):
    """All ranks' server addresses, indexed by rank."""
    if not topo.distributed:
        return [addr]
    out = [None] * topo.world_size
    dist.all_gather_object(out, addr)
    return out


def gather_objects(obj, topo):
    """Every rank's `obj` (picklable), indexed by rank, on every rank."""
    if not topo.distributed:
        return [obj]
    out = [None] * topo.world_size
    dist.all_gather_object(out, obj)
    return out


def ring_peer(topo, hop=1):
    return (topo.rank + hop) % topo.world_size


def destroy(topo):
    if topo.distributed and dist.is_initialized():
        dist.destroy_process_group()
