"""Batched snappy decompression on the GPU (``gpu/snappy_kernels.hip``):
the device half of the snappy body codec. Each input is an independent
raw snappy stream of at most 64 KiB uncompressed (``snappy_compress_blocks``
produces exactly that framing on the host); one wave64 workgroup rebuilds
one block in LDS and streams it to HBM."""
import torch

from ..native import native
from ._common import require_gpu_tensor, stream_handle

MAX_BLOCK = 65536


def snappy_compress_blocks(data, block=MAX_BLOCK):
    """Host: split bytes into <= block-sized pieces, each an independent
    snappy stream. Returns (list_of_compressed_bytes, list_of_raw_lengths)."""
    if block > MAX_BLOCK:
        raise ValueError("block must be <= %d" % MAX_BLOCK)
    comp, lens = [], []
    for off in range(0, len(data), block):
        piece = bytes(data[off:off + block])
        comp.append(native.snappy_compress(piece))
        lens.append(len(piece))
    return comp, lens


def snappy_decompress(packed, offsets, sizes, out_sizes, out=None):
    """Decompress many snappy blocks in one launch.

    packed:    uint8 device tensor holding all compressed blocks
    offsets:   start of each block in ``packed`` (python ints)
    sizes:     compressed size of each block
    out_sizes: uncompressed size of each block (<= 64 KiB)
    out:       optional uint8 device tensor of sum(out_sizes) bytes
    Returns the concatenated uncompressed bytes as a uint8 device tensor.
    """
    require_gpu_tensor(packed, "packed")
    if packed.dtype != torch.uint8:
        raise TypeError("packed must be uint8")
    n = len(offsets)
    if not (len(sizes) == n == len(out_sizes)):
        raise ValueError("offsets/sizes/out_sizes length mismatch")
    dev = packed.device
    total = int(sum(out_sizes))
    if out is None:
        out = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
    elif out.numel() < total:
        raise ValueError("out too small")
    base_in, base_out = packed.data_ptr(), out.data_ptr()
    jobs, pos = [], 0
    for o, s, u in zip(offsets, sizes, out_sizes):
        if u > MAX_BLOCK or o + s > packed.numel():
            raise ValueError("block out of range or larger than 64 KiB")
        jobs += [base_in + int(o), base_out + pos, int(s), int(u)]
        pos += int(u)
    jobs_dev = torch.tensor(jobs, dtype=torch.int64).to(dev)
    meta = torch.zeros(2 * max(n, 1), dtype=torch.int32, device=dev)  # [out_len..., err...]
    with torch.cuda.device(dev):
        native.gpu.snappy_decompress_launch(jobs_dev.data_ptr(), n, meta.data_ptr(), meta.data_ptr() + 4 * n,
                                            stream_handle(dev))
    m = meta.cpu().tolist()
    errs = m[n:2 * n]
    if any(errs):
        bad = [i for i, e in enumerate(errs) if e]
        raise ValueError("malformed snappy block(s) %s (codes %s)" % (bad[:8], [errs[i] for i in bad[:8]]))
    if m[:n] != [int(u) for u in out_sizes]:
        raise ValueError("decoded sizes differ from the expected sizes")
    return out[:total]
