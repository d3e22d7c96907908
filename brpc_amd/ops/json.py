"""JSON structural index on the GPU: the stage-1 tokenizer pass of
http+json bodies (the reference parses them on the CPU through rapidjson,
src/json2pb/json_to_pb.cpp). Returns the byte offsets of every unescaped
quote and of every ``{ } [ ] : ,`` outside strings, in order."""
import torch

from ..native import native
from ._common import require_gpu_tensor, stream_handle

_STRUCTURAL = frozenset(b"{}[]:,")


def json_index(buf, max_positions=None):
    """uint8 device tensor of JSON text -> int64 device tensor of positions.

    Raises ValueError when a string is left open at the end of the input."""
    require_gpu_tensor(buf, "buf")
    if buf.dtype != torch.uint8:
        raise TypeError("buf must be uint8")
    n = buf.numel()
    if n >= 1 << 32:
        raise ValueError("json_index handles inputs below 4 GiB")
    dev = buf.device
    cap = n if max_positions is None else int(max_positions)
    out = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
    meta = torch.zeros(2, dtype=torch.int64, device=dev)  # [count, err]
    scratch = torch.empty(native.gpu.json_index_scratch_bytes(max(n, 1)), dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        native.gpu.json_index_launch(buf.data_ptr(), n, out.data_ptr(), cap, meta.data_ptr(), meta.data_ptr() + 8,
                                     scratch.data_ptr(), stream_handle(dev))
    count, err = meta.tolist()
    err &= 0xFFFFFFFF
    if err & 1:
        raise ValueError("unterminated JSON string")
    if err & 2:
        raise ValueError("more than %d structural positions (found %d)" % (cap, count))
    return out[:count].to(torch.int64)


def json_index_host(data):
    """Pure-python reference of json_index (for tests): (positions, open).

    Like the kernel, a backslash escapes the next byte wherever it stands
    (outside strings it is invalid JSON either way)."""
    out, in_str, esc = [], False, False
    for i, c in enumerate(bytes(data)):
        escaped, esc = esc, (c == 0x5C and not esc)
        if c == 0x22 and not escaped:
            in_str = not in_str
            out.append(i)
        elif not in_str and c in _STRUCTURAL:
            out.append(i)
    return out, in_str
