"""CRC32C (Castagnoli) of device buffers — the checksum carried by
RpcMeta.device_payload (the reference checksums on the CPU only:
src/butil/crc32c.cc)."""
import torch

from ..native import native
from ._common import nbytes, require_gpu_tensor, stream_handle


def crc32c_batch(tensors):
    """Standard CRC32C of the raw bytes of each tensor, one kernel launch per
    32 tensors. Returns an int64 tensor (values in [0, 2^32)) on the device,
    stream-ordered with the current torch stream."""
    if not tensors:
        raise ValueError("empty batch")
    dev = tensors[0].device
    for t in tensors:
        require_gpu_tensor(t)
        if t.device != dev:
            raise ValueError("all tensors must be on one device")
    out = torch.empty(len(tensors), dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        native.gpu.crc32c_launch([t.data_ptr() for t in tensors], [nbytes(t) for t in tensors],
                                 out.data_ptr(), stream_handle(dev))
    return out.to(torch.int64) & 0xFFFFFFFF


def crc32c(t):
    """CRC32C of one device tensor's bytes, as a Python int (synchronises)."""
    return int(crc32c_batch([t])[0].item())


def crc32c_host(data):
    """Host CRC32C (SSE4.2) of bytes-like data — the CPU reference."""
    return native.crc32c(bytes(data))
