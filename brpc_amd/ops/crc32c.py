"""CRC32C (Castagnoli) of device buffers — the checksum carried by
RpcMeta.device_payload (the reference checksums on the CPU only:
src/butil/crc32c.cc). The default kernel computes the CRC as a GF(2)
matrix product on the int8 matrix cores (see csrc/gpu/kernels.hip); the
"lds" implementation (slicing-by-8 tables in LDS) is kept as an independent
cross-check."""
import torch

from ..native import native
from ._common import nbytes, require_gpu_tensor, stream_handle


def _segments_launch(starts, lens, total, maxlen, dev):
    nseg = starts.numel()
    out = torch.empty(nseg, dtype=torch.int32, device=dev)
    scratch = torch.empty(native.gpu.crc32c_scratch_bytes(nseg), dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        native.gpu.crc32c_segments_launch(starts.data_ptr(), lens.data_ptr(), nseg, int(total), int(maxlen),
                                          out.data_ptr(), scratch.data_ptr(), stream_handle(dev))
    return out.to(torch.int64) & 0xFFFFFFFF


def crc32c_batch(tensors, impl="mfma"):
    """Standard CRC32C of the raw bytes of each tensor in one launch.
    Returns an int64 tensor (values in [0, 2^32)) on the device,
    stream-ordered with the current torch stream."""
    if not tensors:
        raise ValueError("empty batch")
    dev = tensors[0].device
    for t in tensors:
        require_gpu_tensor(t)
        if t.device != dev:
            raise ValueError("all tensors must be on one device")
    sizes = [nbytes(t) for t in tensors]
    if impl == "lds":
        out = torch.empty(len(tensors), dtype=torch.int32, device=dev)
        with torch.cuda.device(dev):
            native.gpu.crc32c_lds_launch([t.data_ptr() for t in tensors], sizes, out.data_ptr(), stream_handle(dev))
        return out.to(torch.int64) & 0xFFFFFFFF
    if impl != "mfma":
        raise ValueError("impl must be 'mfma' or 'lds'")
    desc = torch.tensor([[t.data_ptr() for t in tensors], sizes], dtype=torch.int64).to(dev, non_blocking=True)
    return _segments_launch(desc[0], desc[1], sum(sizes), max(sizes), dev)


def crc32c_packed(buf, offsets):
    """CRC32C of each message packed in one uint8 device buffer:
    message i = buf[offsets[i]:offsets[i+1]] (offsets: int64 device tensor,
    n+1 entries). One launch, no host round trip for the segment table."""
    require_gpu_tensor(buf, "buf")
    require_gpu_tensor(offsets, "offsets")
    if offsets.dtype != torch.int64:
        raise TypeError("offsets must be int64")
    dev = buf.device
    starts = offsets[:-1] + buf.data_ptr()
    lens = offsets[1:] - offsets[:-1]
    return _segments_launch(starts.contiguous(), lens.contiguous(), nbytes(buf), nbytes(buf), dev)


def crc32c(t, impl="mfma"):
    """CRC32C of one device tensor's bytes, as a Python int (synchronises)."""
    return int(crc32c_batch([t], impl=impl)[0].item())


def crc32c_host(data):
    """Host CRC32C (SSE4.2) of bytes-like data — the CPU reference."""
    return native.crc32c(bytes(data))
