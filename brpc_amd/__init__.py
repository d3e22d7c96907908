"""brpc_amd — an MI355X-native RPC framework with bRPC's capabilities.

The engine is native C++ (``brpc_amd/lib/libmrpc.so``: M:N fiber runtime,
sockets, protocols, Channel/Server/Controller, metrics, press) plus
hand-written CDNA4 HIP kernels for the device data path. This package is the
Python face used by ``bench.py``, the tests and torch-side code:

* :mod:`brpc_amd.native`   — the pybind11 extension (loaded in-tree; fails
  loudly when missing)
* :mod:`brpc_amd.ops`      — device ops on torch tensors (CRC32C, packed
  varint codec, batched copy)
* :mod:`brpc_amd.parallel` — one-process-per-GPU topology over
  torch.distributed (RCCL) and peer address exchange
* :mod:`brpc_amd.models`   — benchmark/service workloads (echo, streaming)
* :mod:`brpc_amd.utils`    — build helpers, flags and metrics access
"""
from .native import native, Server, Channel, Press  # noqa: F401

__version__ = "0.1.0"
