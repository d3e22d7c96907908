"""Batched protobuf wire scan on the GPU (``gpu/pb_kernels.hip``): decode the
top-level fields of many small serialized messages (RpcMeta-sized) packed in
one device buffer, one lane per message, one launch."""
import torch

from ..native import native
from ._common import require_gpu_tensor, stream_handle

WIRE_VARINT, WIRE_FIXED64, WIRE_LEN, WIRE_FIXED32 = 0, 1, 2, 5
ERRORS = {-1: "truncated or malformed", -2: "too many fields", -3: "field number 0", -4: "unsupported wire type",
          -5: "offsets outside the buffer or descending"}


def pb_scan(buf, offsets, max_fields=16):
    """buf: uint8 device tensor; offsets: int64 device tensor of n+1 message
    boundaries. Returns (fields, nfields): fields is an int64 (n, max_fields,
    2) tensor of [tag, value] rows (tag = field << 3 | wire; value = varint,
    fixed bits, or offset << 32 | length for wire 2, offset relative to the
    message), nfields an int32 (n,) tensor of field counts (negative = error,
    see ERRORS)."""
    require_gpu_tensor(buf, "buf")
    require_gpu_tensor(offsets, "offsets")
    if buf.dtype != torch.uint8 or offsets.dtype != torch.int64:
        raise TypeError("buf must be uint8 and offsets int64")
    if offsets.device != buf.device:
        raise ValueError("offsets must live on the same device as buf (%s vs %s)" % (offsets.device, buf.device))
    if not buf.is_contiguous() or not offsets.is_contiguous():
        raise ValueError("buf and offsets must be contiguous")
    n = offsets.numel() - 1
    dev = buf.device
    fields = torch.zeros((max(n, 1), max_fields, 2), dtype=torch.int64, device=dev)
    nfields = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)
    if n > 0:
        with torch.cuda.device(dev):
            # the kernel bounds every message by buf.numel() (code -5)
            native.gpu.pb_scan_launch(buf.data_ptr(), buf.numel(), offsets.data_ptr(), n, int(max_fields),
                                      fields.data_ptr(), nfields.data_ptr(), stream_handle(dev))
    return fields[:n], nfields[:n]


def pb_scan_host(msg, max_fields=16):
    """Pure-python reference of one message's scan (tests)."""
    out, p = [], 0

    def varint():
        nonlocal p
        v, shift = 0, 0
        while True:
            if p >= len(msg) or shift >= 70:
                raise ValueError("truncated")
            c = msg[p]
            p += 1
            v |= (c & 0x7F) << shift
            if not c & 0x80:
                return v
            shift += 7

    while p < len(msg):
        tag = varint()
        field, wire = tag >> 3, tag & 7
        if field == 0:
            return out, -3
        if wire == 0:
            val = varint()
        elif wire in (1, 5):
            nb = 8 if wire == 1 else 4
            if len(msg) - p < nb:
                return out, -1
            val = int.from_bytes(msg[p:p + nb], "little")
            p += nb
        elif wire == 2:
            ln = varint()
            if ln > len(msg) - p:
                return out, -1
            val = (p << 32) | ln
            p += ln
        else:
            return out, -4
        if len(out) >= max_fields:
            return out, -2
        out.append((tag, val))
    return out, len(out)
