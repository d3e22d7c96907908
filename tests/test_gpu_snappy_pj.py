"""The data-parallel snappy compressor (snappy_kernels.hip compress_wave_pj,
-gpu_snappy_compress_pj): every position's candidate and match length at
once, the greedy element chain by pointer doubling. Every block it writes is
a standard raw snappy stream (the host codec base/snappy.cc decodes it, and
so does the device decoder), for blocks up to 4 KiB, on incompressible,
run-heavy, mixed, constant and log-text bodies and at the edge sizes of the
parse (no 4-byte position, one element, block ends inside a match); larger
blocks fall back to the per-lane-slice compressor. On text its output is
smaller than the slice compressor's (matches cross the old slice ends)."""
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
def _pj_on(native):
    old = native.get_flag("gpu_snappy_compress_pj")
    native.set_flag("gpu_snappy_compress_pj", "true")
    yield
    native.set_flag("gpu_snappy_compress_pj", old)
    native.set_flag("device_payload_block_kb", "2")


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
        return b"q" * n
    if kind == "period":  # short periods: overlapping copies, offsets 1..7
        p = bytes(rnd.getrandbits(8) for _ in range(rnd.randint(1, 7)))
        return (p * (n // len(p) + 1))[:n]
    from brpc_amd import native as nat
    return nat.echo_body("text", n)


def _compress(native, data, block):
    from brpc_amd.ops import snappy_compress, snappy_decompress
    dev = torch.device("cuda", 0)
    t = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    packed, offs, sizes, raw = snappy_compress(t, block=block)
    host = packed.cpu().numpy().tobytes()
    back = b"".join(native.snappy_uncompress(host[o:o + s]) for o, s in zip(offs, sizes))
    assert back == data
    out = snappy_decompress(packed, offs, sizes, raw)
    assert out.cpu().numpy().tobytes() == data
    return sum(sizes)


KINDS = ["random", "runs", "mixed", "const", "period", "text"]


@pytest.mark.parametrize("block", [1024, 2048, 4096])
@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("size", [1, 3, 4, 5, 6, 7, 8, 63, 64, 65, 1000, 1023, 2049, 4095, 4096, 4097, 65539])
def test_pj_blocks_are_standard_snappy(native, block, kind, size):
    _compress(native, _corpus(kind, size, size * 13 + block + len(kind)), block)


@pytest.mark.parametrize("block", [2048, 4096])
def test_pj_beats_lane_slices_on_text(native, block):
    data = _corpus("text", 1 << 18, 5)
    pj = _compress(native, data, block)
    native.set_flag("gpu_snappy_compress_pj", "false")
    slices = _compress(native, data, block)
    assert pj < slices, (pj, slices)
    assert len(data) / pj > (2.1 if block == 2048 else 2.3), len(data) / pj


def test_pj_falls_back_above_4k_blocks(native):
    data = _corpus("mixed", 100000, 3)
    _compress(native, data, 8192)
    _compress(native, data, 65536)


@pytest.mark.parametrize("kb", [1, 2, 4, 8])
@pytest.mark.parametrize("kind", ["text", "random", "const", "mixed"])
def test_pj_in_the_device_codec_batch(native, kb, kind):
    """The codec batch's one-launch kernel (codec_waves_kernel<.., kPj>):
    payload blocks compressed on the device decode on the host and on the
    device."""
    native.set_flag("device_payload_block_kb", str(kb))
    dev = torch.device("cuda", 0)
    data = _corpus(kind, 70001, kb * 7 + len(kind))
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
    err, _, _ = native.gpu.device_snappy_decode(region.data_ptr(), region.numel(), ulen, stride, clen,
                                                out.data_ptr(), len(data), False, 0)
    assert err == 0
    assert out.cpu().numpy().tobytes() == data
