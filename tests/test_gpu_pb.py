"""GPU protobuf wire scan (gpu/pb_kernels.hip) against a pure-python
reference decoder of the same bytes: random messages mixing varints (up to
full 64-bit), fixed32/64 and length-delimited fields, many messages per
launch, and every malformed-input code."""
import random

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

M64 = (1 << 64) - 1


@pytest.fixture(scope="module")
def dev():
    from brpc_amd import native
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    assert native.gpu.device_count() > 0
    return torch.device("cuda", 0)


def _varint(v):
    out = bytearray()
    v &= M64
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _message(rnd, nfields):
    out = bytearray()
    for _ in range(nfields):
        field = rnd.choice([1, 2, 3, 15, 16, 100, 2047, 536870911])
        wire = rnd.choice([0, 0, 1, 2, 2, 5])
        out += _varint(field << 3 | wire)
        if wire == 0:
            out += _varint(rnd.choice([0, 1, 127, 128, 300, rnd.getrandbits(32), rnd.getrandbits(64), M64]))
        elif wire == 1:
            out += rnd.getrandbits(64).to_bytes(8, "little")
        elif wire == 5:
            out += rnd.getrandbits(32).to_bytes(4, "little")
        else:
            body = bytes(rnd.getrandbits(8) for _ in range(rnd.choice([0, 1, 5, 40, 200])))
            out += _varint(len(body)) + body
    return bytes(out)


def _run(dev, msgs, max_fields=16):
    from brpc_amd.ops import pb_scan
    offs = [0]
    for m in msgs:
        offs.append(offs[-1] + len(m))
    data = b"".join(msgs) or b"\0"
    buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    o = torch.tensor(offs, dtype=torch.int64, device=dev)
    fields, nfields = pb_scan(buf, o, max_fields)
    return fields.cpu().tolist(), nfields.cpu().tolist()


def test_pb_scan_matches_reference(dev):
    from brpc_amd.ops.pb import pb_scan_host
    rnd = random.Random(7)
    msgs = [_message(rnd, rnd.randint(0, 12)) for _ in range(5000)]
    fields, nfields = _run(dev, msgs)
    for i, m in enumerate(msgs):
        want, code = pb_scan_host(m)
        assert nfields[i] == code, (i, nfields[i], code)
        got = [(t & M64, v & M64) for t, v in fields[i][:code]]
        assert got == want, i


def test_pb_scan_error_codes(dev):
    msgs = [
        b"\x08\x96",                     # truncated varint value
        b"\x0a\x05abc",                  # length beyond the message
        b"\x00\x01",                     # field number 0
        b"\x0b\x0c",                     # group (wire 3)
        b"".join(_varint(1 << 3) + b"\x01" for _ in range(5)),  # 5 fields, max 4
        b"\x08" + b"\xff" * 9 + b"\x02",  # varint overflowing 64 bits
        b"",                             # empty message: 0 fields
        b"\x08\x01",                     # ok: one field
    ]
    _, nfields = _run(dev, msgs, max_fields=4)
    assert nfields == [-1, -1, -3, -4, -2, -1, 0, 1]


def test_pb_scan_rejects_bad_offsets(dev):
    """the offset table is never trusted — messages past the end of
    the buffer or with descending bounds report -5 and are not read."""
    from brpc_amd.ops import pb_scan
    data = b"\x08\x01\x10\x02"
    buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    o = torch.tensor([0, 2, 4, 1 << 40, 3, 2], dtype=torch.int64, device=dev)
    _, nfields = pb_scan(buf, o, 4)
    assert nfields.cpu().tolist() == [1, 1, -5, -5, -5]
    with pytest.raises((ValueError, TypeError)):
        pb_scan(buf, o.cpu(), 4)  # offsets on another device than buf
