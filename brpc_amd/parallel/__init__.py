"""One process per GPU over torch.distributed (backend "nccl" = RCCL on
ROCm): rank topology, peer address exchange and cross-rank reductions used
by the benchmarks and by the xGMI device transport's handshake."""
from .topology import (Topology, init_distributed, exchange_addresses, ring_peer, barrier,  # noqa: F401
                       allreduce_max, allreduce_sum, destroy, gather_objects)
from .rccl import (init_rccl_plane, set_rccl_min_bytes, rccl_stats, shutdown_rccl_plane,  # noqa: F401,E402
                   stub_library)
