"""One-launch gather/scatter of many byte ranges (Buf blocks -> HBM)."""
from ..native import native
from ._common import nbytes, require_gpu_tensor, stream_handle


def batched_copy(srcs, dsts):
    """dsts[i][:] = srcs[i][:] (byte copies) in one kernel launch per 32 pairs."""
    if len(srcs) != len(dsts):
        raise ValueError("srcs/dsts length mismatch")
    for s, d in zip(srcs, dsts):
        require_gpu_tensor(s, "src")
        require_gpu_tensor(d, "dst")
        if nbytes(d) < nbytes(s):
            raise ValueError("destination smaller than source")
    if not srcs:
        return
    dev = srcs[0].device
    native.gpu.batched_copy_launch([s.data_ptr() for s in srcs], [d.data_ptr() for d in dsts],
                                   [nbytes(s) for s in srcs], stream_handle(dev))


def batched_copy_crc32c(srcs, dsts, mfma=True):
    """Fused: dsts[i][:] = srcs[i][:] and returns the standard CRC32C of each
    source (int64 device tensor) — one read of the bytes (the pull kernel of
    the xGMI transport's verified receives). mfma: the CRC runs on the matrix
    cores (the default; False: the byte-table kernel)."""
    import torch
    if len(srcs) != len(dsts):
        raise ValueError("srcs/dsts length mismatch")
    for s, d in zip(srcs, dsts):
        require_gpu_tensor(s, "src")
        require_gpu_tensor(d, "dst")
        if nbytes(d) < nbytes(s):
            raise ValueError("destination smaller than source")
    if not srcs:
        return None
    dev = srcs[0].device
    # no zeroing needed: the kernel stores each finished CRC (fold_segment_crc)
    out = torch.empty(len(srcs), dtype=torch.int32, device=dev)
    native.gpu.batched_copy_crc32c_launch([s.data_ptr() for s in srcs], [d.data_ptr() for d in dsts],
                                          [nbytes(s) for s in srcs], out.data_ptr(), stream_handle(dev), mfma)
    return out.to(torch.int64) & 0xFFFFFFFF
