"""One-launch codec batches behind the device payload codec
(codec_waves_kernel, snappy_kernels.hip: one wave per block/piece). Every
block it writes is a standard raw snappy stream (the host codec decodes it),
the device decoder rebuilds the payload from it, text keeps the ratio the
bench leg is quoted at, the last piece of a message scans its fields, and
malformed pieces are refused without hanging. Numerics against the host
snappy codec (base/snappy.cc) and numpy byte equality."""
import random

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from brpc_amd import native as n
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    assert n.gpu.device_count() > 0
    return n


@pytest.fixture(autouse=True)
def _restore_flags(native):
    native.set_flag("codec_fused", "true")
    yield
    native.set_flag("device_payload_block_kb", "2")
    native.set_flag("codec_fused", "true")
    native.set_flag("codec_fused_scan_in_kernel", "false")


def _corpus(kind, n, seed):
    rnd = random.Random(seed)
    if kind == "random":
        return bytes(rnd.getrandbits(8) for _ in range(n))
    if kind == "runs":
        out = bytearray()
        while len(out) < n:
            out += bytes([rnd.getrandbits(8)]) * rnd.randint(1, 300)
        return bytes(out[:n])
    if kind == "mixed":
        out = bytearray(rnd.getrandbits(8) for _ in range(64))
        while len(out) < n:
            if rnd.random() < 0.5:
                s = rnd.randrange(len(out))
                out += out[s:s + rnd.randint(4, 200)]
            else:
                out += bytes(rnd.getrandbits(8) for _ in range(rnd.randint(1, 40)))
        return bytes(out[:n])
    if kind == "const":
        return b"x" * n
    from brpc_amd import native as nat
    return nat.echo_body("text", n)


def _varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _roundtrip(native, data, scan=False):
    dev = torch.device("cuda", 0)
    src = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    ulen, stride, nblocks = native.gpu.device_snappy_layout(len(data))
    region = torch.zeros(stride * nblocks, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    clen = native.gpu.device_snappy_encode(src.data_ptr(), len(data), region.data_ptr(), 0)
    host = region.cpu().numpy().tobytes()
    for i, c in enumerate(clen):
        assert 0 < c <= stride
        assert native.snappy_uncompress(host[i * stride:i * stride + c]) == data[i * ulen:(i + 1) * ulen], i
    out = torch.zeros(len(data), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    err, nf, fields = native.gpu.device_snappy_decode(region.data_ptr(), region.numel(), ulen, stride, clen,
                                                      out.data_ptr(), len(data), scan, 0)
    assert err == 0
    assert out.cpu().numpy().tobytes() == data
    return sum(clen), nf, fields


@pytest.mark.parametrize("kb", [1, 2, 4, 8])
@pytest.mark.parametrize("kind", ["text", "random", "runs", "mixed", "const"])
@pytest.mark.parametrize("size", [1, 5, 63, 64, 65, 4095, 4096, 4097, 65536, 100003])
def test_fused_blocks_round_trip(native, kb, kind, size):
    native.set_flag("device_payload_block_kb", str(kb))
    before = native.gpu.codec_batch_stats()["fused_launches"]
    _roundtrip(native, _corpus(kind, size, size * 31 + kb))
    assert native.gpu.codec_batch_stats()["fused_launches"] - before >= 2  # the encode and the decode


@pytest.mark.parametrize("kb,floor", [(2, 1.9), (4, 2.1)])
def test_fused_text_ratio_and_per_stage_agree(native, kb, floor):
    """Text keeps the ratio the device leg is quoted at, and the one-launch
    batch writes the same bytes as the per-stage launches."""
    native.set_flag("device_payload_block_kb", str(kb))
    data = _corpus("text", 1 << 18, 7)
    fused, _, _ = _roundtrip(native, data)
    native.set_flag("codec_fused", "false")
    staged, _, _ = _roundtrip(native, data)
    assert fused == staged
    assert len(data) / fused >= floor, len(data) / fused


@pytest.mark.parametrize("in_kernel", [False, True])
def test_fused_scan_runs_after_the_last_piece(native, in_kernel):
    """The message's field table: by the wave that finished its last piece
    (in_kernel) or by the pb-scan launch after the batch."""
    native.set_flag("codec_fused_scan_in_kernel", "true" if in_kernel else "false")
    native.set_flag("device_payload_block_kb", "4")
    body = native.echo_body("text", 50000)
    msg = bytes([0x0A]) + _varint(len(body)) + body + bytes([0x18, 0x01])
    for _ in range(3):  # the group counters reset for the next launch
        _, nf, fields = _roundtrip(native, msg, scan=True)
        off = 1 + len(_varint(len(body)))
        assert nf == 2
        assert fields[0] == (1 << 3) | 2 and fields[1] == (off << 32) | len(body)
        assert fields[2] == (3 << 3) | 0 and fields[3] == 1


@pytest.mark.parametrize("seed", range(6))
def test_fused_decoder_refuses_corrupt_pieces(native, seed):
    """Random byte damage in a compressed block: the decode reports an
    error or (if the damage left a valid stream) returns bytes; it never
    hangs or writes outside its block."""
    native.set_flag("device_payload_block_kb", "4")
    dev = torch.device("cuda", 0)
    data = _corpus("mixed", 40000, seed)
    src = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    ulen, stride, nblocks = native.gpu.device_snappy_layout(len(data))
    region = torch.zeros(stride * nblocks, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    clen = native.gpu.device_snappy_encode(src.data_ptr(), len(data), region.data_ptr(), 0)
    host = bytearray(region.cpu().numpy().tobytes())
    rnd = random.Random(seed)
    hits = 0
    for i, c in enumerate(clen):
        h = len(_varint(min(ulen, len(data) - i * ulen)))
        for _ in range(1 + seed):
            k = i * stride + rnd.randrange(h, c)
            host[k] ^= 1 << rnd.randrange(8)
            hits += 1
    region2 = torch.frombuffer(host, dtype=torch.uint8).to(dev)
    # a guard band after the output catches writes past the payload
    out = torch.full((len(data) + 4096,), 0xA5, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    err, _, _ = native.gpu.device_snappy_decode(region2.data_ptr(), region2.numel(), ulen, stride, clen,
                                                out.data_ptr(), len(data), False, 0)
    assert err in (0, 2)
    tail = out[len(data):].cpu().numpy()
    assert (tail == 0xA5).all()
    assert hits > 0
