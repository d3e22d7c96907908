"""Batched snappy compression and decompression on the GPU
(``gpu/snappy_kernels.hip``): the device half of the snappy body codec.
Each block is an independent raw snappy stream of at most 64 KiB
uncompressed (``snappy_compress_blocks`` produces that framing on the host,
``snappy_compress`` on the device); one wave64 workgroup owns one block.
Both directions interoperate with the host codec (``native.snappy_*``)."""
import torch

from ..native import native
from ._common import require_gpu_tensor, stream_handle

MAX_BLOCK = 65536
# Default device framing block: 32 KiB blocks decode ~1.75x faster than
# 64 KiB ones (LDS per wave halves: 5 waves per CU instead of 2) for ~0.2%
# larger output (profiles/kernels_r1_microbench.jsonl).
DEFAULT_BLOCK = 32768


def snappy_compress_blocks(data, block=DEFAULT_BLOCK):
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
    max_ulen = max([int(u) for u in out_sizes] + [1])
    with torch.cuda.device(dev):
        native.gpu.snappy_decompress_launch(jobs_dev.data_ptr(), n, max_ulen, meta.data_ptr(),
                                            meta.data_ptr() + 4 * n, stream_handle(dev))
    m = meta.cpu().tolist()
    errs = m[n:2 * n]
    if any(errs):
        bad = [i for i, e in enumerate(errs) if e]
        raise ValueError("malformed snappy block(s) %s (codes %s)" % (bad[:8], [errs[i] for i in bad[:8]]))
    if m[:n] != [int(u) for u in out_sizes]:
        raise ValueError("decoded sizes differ from the expected sizes")
    return out[:total]


def snappy_decompress_streams(packed, offsets, sizes, out_sizes, piece_limit=4096, out=None):
    """Decompress whole raw snappy streams of any length: the device cuts
    each stream into self-contained pieces (``snappy_split_kernel``, one wave
    walking the element headers; <= piece_limit uncompressed bytes, else the
    64 KiB fragments of CPU encoders) and decodes the pieces in parallel; no
    host tag walk. Same arguments as ``snappy_decompress`` minus the 64 KiB
    limit. Raises ValueError naming the streams the device refused."""
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
    if n == 0:
        return out[:0]
    base_in, base_out = packed.data_ptr(), out.data_ptr()
    rows, pos, first = [], 0, 0
    for o, s, u in zip(offsets, sizes, out_sizes):
        if o + s > packed.numel() or s >= 1 << 32 or u >= 1 << 32:
            raise ValueError("stream out of range")
        mp = int(native.gpu.snappy_max_pieces(int(u), piece_limit))
        rows += [base_in + int(o), base_out + pos, int(s) | (int(u) << 32), first | (mp << 32)]
        pos += int(u)
        first += mp
    streams_dev = torch.tensor(rows, dtype=torch.int64).to(dev)
    pieces = torch.empty(first * int(native.gpu.snappy_piece_bytes()), dtype=torch.uint8, device=dev)
    errs = torch.full((n + first,), -1, dtype=torch.int32, device=dev)  # [stream codes..., piece codes...]
    small = min(piece_limit, MAX_BLOCK)
    with torch.cuda.device(dev):
        h = stream_handle(dev)
        native.gpu.snappy_split_launch(streams_dev.data_ptr(), n, small, pieces.data_ptr(), errs.data_ptr(), h)
        native.gpu.snappy_decompress_pieces_launch(pieces.data_ptr(), first, 0, small, errs.data_ptr() + 4 * n, h)
        if small < MAX_BLOCK:
            native.gpu.snappy_decompress_pieces_launch(pieces.data_ptr(), first, small, MAX_BLOCK,
                                                       errs.data_ptr() + 4 * n, h)
    e = errs.cpu().tolist()
    bad, first = [], 0
    for i, u in enumerate(out_sizes):
        mp = int(native.gpu.snappy_max_pieces(int(u), piece_limit))
        code = e[i] or next((c for c in e[n + first:n + first + mp] if c), 0)
        if code:
            bad.append((i, code))
        first += mp
    if bad:
        raise ValueError("malformed or uncuttable snappy stream(s) %s" % bad[:8])
    return out[:total]


def snappy_compress(data, block=DEFAULT_BLOCK, compact=True):
    """Compress a uint8 device tensor on the GPU as independent snappy blocks
    of ``block`` bytes (the last one may be shorter), one launch for all.

    Returns (packed, offsets, comp_sizes, raw_sizes): ``packed`` is a uint8
    device tensor holding the compressed blocks back to back when ``compact``
    (else in fixed-stride slots), ready for ``snappy_decompress``; every block
    also decodes with the host codec."""
    require_gpu_tensor(data, "data")
    if data.dtype != torch.uint8:
        raise TypeError("data must be uint8")
    if not 0 < block <= MAX_BLOCK:
        raise ValueError("block must be in (0, %d]" % MAX_BLOCK)
    dev = data.device
    total = data.numel()
    raw = [min(block, total - o) for o in range(0, total, block)]
    n = len(raw)
    if n == 0:
        return torch.zeros(0, dtype=torch.uint8, device=dev), [], [], []
    cap = (int(native.gpu.snappy_max_compressed_length(block)) + 15) & ~15
    slots = torch.empty(n * cap, dtype=torch.uint8, device=dev)
    scratch = torch.empty(n * int(native.gpu.snappy_compress_scratch_per_block()), dtype=torch.uint8, device=dev)
    base_in, base_out = data.data_ptr(), slots.data_ptr()
    jobs = []
    for i, r in enumerate(raw):
        jobs += [base_in + i * block, base_out + i * cap, r, cap]
    jobs_dev = torch.tensor(jobs, dtype=torch.int64).to(dev)
    meta = torch.zeros(2 * n, dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        native.gpu.snappy_compress_launch(jobs_dev.data_ptr(), n, max(raw), scratch.data_ptr(), meta.data_ptr(),
                                          meta.data_ptr() + 4 * n, stream_handle(dev))
    m = meta.cpu().tolist()
    if any(m[n:]):
        raise RuntimeError("snappy_compress failed for blocks %s" % [i for i, e in enumerate(m[n:]) if e][:8])
    sizes = m[:n]
    if not compact:
        return slots, [i * cap for i in range(n)], sizes, raw
    packed = torch.cat([slots[i * cap:i * cap + sz] for i, sz in enumerate(sizes)])
    offs, pos = [], 0
    for sz in sizes:
        offs.append(pos)
        pos += sz
    return packed, offs, sizes, raw
