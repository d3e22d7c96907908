"""RCCL data plane for RPC payloads (native side: csrc/gpu/rccl_plane.h).

Every rank of a torchrun job calls :func:`init_rccl_plane` once, before it
opens connections: rank 0 generates the RCCL unique id, the process group
broadcasts it, and each rank joins one communicator on its GPU. Connections
between ranks of the plane then announce their rank in the xGMI hello, and
device payload blocks of at least ``-rccl_min_bytes`` travel by
ncclSend/ncclRecv (sequence numbers in the RPC meta) instead of xGMI
lending. The plane replaces the reference's RDMA zero-copy path
(src/brpc/rdma/rdma_endpoint.cpp:771-895) for large payloads.
"""
import torch.distributed as dist

from .. import native


def init_rccl_plane(topo, min_bytes=None):
    """Join the job's RCCL plane on ``topo.device``. ``min_bytes`` sets the
    payload threshold now (None leaves the flag alone: the default never
    uses the plane). Returns True when the plane is up; a CPU topology has
    no plane and returns False."""
    if topo.device < 0:
        return False
    if topo.world_size > 1:
        box = [native.gpu.rccl_unique_id() if topo.rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        uid = box[0]
    else:
        uid = native.gpu.rccl_unique_id()
    native.gpu.rccl_init(topo.rank, topo.world_size, uid, topo.device)
    if min_bytes is not None:
        set_rccl_min_bytes(min_bytes)
    return native.gpu.rccl_active()


def set_rccl_min_bytes(n):
    """Payload threshold (reloadable); ``None`` or <=0 turns the plane off
    for new payloads."""
    native.set_flag("rccl_min_bytes", str(int(n) if n and n > 0 else 1 << 40))


def rccl_stats():
    return native.gpu.rccl_stats()


def shutdown_rccl_plane():
    native.gpu.rccl_shutdown()
