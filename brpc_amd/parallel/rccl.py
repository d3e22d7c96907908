"""RCCL payload plane for RPC payloads (native side: csrc/gpu/rccl_plane.h).

Every rank of a one-node torchrun job calls :func:`init_rccl_plane` once,
before it opens connections: rank 0 generates the unique id, the process
group broadcasts it, and each rank joins the plane (one communicator, one
stream, numbered rounds). Connections between ranks of the plane then
exchange a plane hello, and attachment payloads of at least
``-rccl_min_bytes`` travel by ncclSend/ncclRecv (sequence numbers in the RPC
meta) instead of xGMI lending. The plane plays the part of the reference's
RDMA zero-copy path (src/brpc/rdma/rdma_endpoint.cpp:771-895, credits at
:505-509).

On CPU-only hosts ``library=stub_library()`` runs the same plane on the stub
RCCL (csrc/tests/stub/fake_rccl.cc: bounded shared-memory FIFOs, one
in-order queue per process) with host-memory payloads, so multi-rank jobs
rehearse the plane with gloo.
"""
import os

import torch.distributed as dist

from .. import native

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def stub_library():
    """Path of the stub RCCL library built by build.py."""
    return os.path.join(_ROOT, "build", "lib", "libfake_rccl.so")


def init_rccl_plane(topo, min_bytes=None, library=None):
    """Join the job's RCCL plane on ``topo.device`` (or on the stub library
    when ``library`` is given). ``min_bytes`` sets the payload threshold now
    (None leaves the flag alone: the default never uses the plane). Returns
    True when the plane is up; a CPU topology without ``library`` has no
    plane and returns False."""
    if library:
        native.set_flag("rccl_library", library)
    elif topo.device < 0:
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
