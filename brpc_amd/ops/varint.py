"""Packed protobuf varints encoded/decoded on the GPU (e.g. token-id
payloads of a `repeated int64 ids = 1 [packed=true]` field), the
device-side half of the pb wire codec."""
import torch

from ..native import native
from ._common import require_gpu_tensor, stream_handle


def varint_decode(buf, zigzag=False, max_values=None):
    """Decode a uint8 device tensor of concatenated varints -> int64 tensor."""
    require_gpu_tensor(buf, "buf")
    if buf.dtype != torch.uint8:
        raise TypeError("buf must be uint8")
    n = buf.numel()
    dev = buf.device
    cap = n if max_values is None else int(max_values)
    out = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
    meta = torch.zeros(2, dtype=torch.int64, device=dev)  # [count, err]
    scratch = torch.empty(native.gpu.varint_scratch_bytes(max(n, 1)), dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        native.gpu.varint_decode_launch(buf.data_ptr(), n, out.data_ptr(), cap, bool(zigzag), meta.data_ptr(),
                                        meta.data_ptr() + 8, scratch.data_ptr(), stream_handle(dev))
    count, err = meta.tolist()
    if err & 0xFFFFFFFF:
        raise ValueError("malformed varint stream (code %d)" % (err & 0xFFFFFFFF))
    return out[:count]


def varint_encode(values, zigzag=False):
    """Encode an int64 device tensor -> uint8 device tensor of varints."""
    require_gpu_tensor(values, "values")
    if values.dtype != torch.int64:
        raise TypeError("values must be int64")
    n = values.numel()
    dev = values.device
    out = torch.empty(max(10 * n, 1), dtype=torch.uint8, device=dev)
    nbytes = torch.zeros(1, dtype=torch.int64, device=dev)
    scratch = torch.empty(native.gpu.varint_scratch_bytes(max(n, 1)), dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        native.gpu.varint_encode_launch(values.data_ptr(), n, bool(zigzag), out.data_ptr(), nbytes.data_ptr(),
                                        scratch.data_ptr(), stream_handle(dev))
    return out[: int(nbytes.item())]


def varint_encode_host(values, zigzag=False):
    """Pure-python reference encoder (for tests)."""
    out = bytearray()
    for v in values:
        v = int(v)
        if zigzag:
            v = (v << 1) ^ (v >> 63)
        v &= (1 << 64) - 1
        while v >= 0x80:
            out.append((v & 0x7F) | 0x80)
            v >>= 7
        out.append(v)
    return bytes(out)


def varint_decode_host(data, zigzag=False):
    out, v, shift = [], 0, 0
    for b in data:
        v |= (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            v &= (1 << 64) - 1
            if zigzag:
                v = (v >> 1) ^ -(v & 1)
            elif v >= 1 << 63:
                v -= 1 << 64
            out.append(v)
            v, shift = 0, 0
    return out
