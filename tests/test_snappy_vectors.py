"""Known-answer snappy streams built by hand from the format description the
reference vendors (src/butil/third_party/snappy/format_description.txt):
the varint preamble (its 64 / 2097150 examples, lines 20-25), literals with
inline and 1-4 byte lengths (2.1), copies with 1-, 2- and 4-byte offsets
(2.2.1-2.2.3), the "xababab" overlapping-copy example (lines 73-77) and the
streams it calls illegal (offset 0, offsets past the output, a leading copy).

Checked against the host codec (base/snappy.cc) on CPU, and against the
GPU decompressor (gpu/snappy_kernels.hip) in the same launch on a GPU box.
These are independent of any compressor, ours included."""
import pytest


def varint(n):
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            return bytes(out)


def lit(data, nbytes=0):
    """Literal element; nbytes=0 inlines len-1 in the tag when it fits,
    otherwise (or when forced) the length takes 1..4 bytes (tag 60..63)."""
    n = len(data) - 1
    if nbytes == 0 and n < 60:
        return bytes([n << 2]) + data
    if nbytes == 0:
        nbytes = 1 if n < 1 << 8 else 2 if n < 1 << 16 else 3 if n < 1 << 24 else 4
    return bytes([(59 + nbytes) << 2]) + n.to_bytes(nbytes, "little") + data


def copy1(length, offset):
    assert 4 <= length <= 11 and offset < 2048
    return bytes([0x01 | ((length - 4) << 2) | ((offset >> 8) << 5), offset & 0xFF])


def copy2(length, offset):
    assert 1 <= length <= 64 and offset < 65536
    return bytes([0x02 | ((length - 1) << 2)]) + offset.to_bytes(2, "little")


def copy4(length, offset):
    assert 1 <= length <= 64
    return bytes([0x03 | ((length - 1) << 2)]) + offset.to_bytes(4, "little")


def stream(ulen, *elements):
    return varint(ulen) + b"".join(elements)


L300 = bytes((i * 7) & 0xFF for i in range(300))

VALID = [
    ("empty", stream(0), b""),
    ("xababab", stream(7, lit(b"xab"), copy1(4, 2)), b"xababab"),  # format_description.txt:75-77
    ("literal_60_inline", stream(60, lit(b"L" * 60)), b"L" * 60),
    ("literal_61_one_byte_len", stream(61, lit(b"M" * 61)), b"M" * 61),
    ("literal_300_two_byte_len", stream(300, lit(L300)), L300),
    ("literal_3_byte_len_nonminimal", stream(100, lit(b"N" * 100, 3)), b"N" * 100),
    ("literal_4_byte_len_nonminimal", stream(5, lit(b"hello", 4)), b"hello"),
    ("copy1_high_offset_bits", stream(311, lit(L300), copy1(11, 300)), L300 + L300[:11]),
    ("copy2_rle_64", stream(68, lit(b"abcd"), copy2(64, 4)), b"abcd" * 17),
    ("copy2_offset_1_run", stream(65, lit(b"z"), copy2(64, 1)), b"z" * 65),
    ("copy4", stream(13, lit(b"xyz"), copy4(10, 3)), b"xyz" + b"xyzxyzxyzx"),
    ("two_literals_in_a_row", stream(6, lit(b"abc"), lit(b"def")), b"abcdef"),  # permitted (2.)
    ("mixed", stream(3 + 8 + 2 + 5, lit(b"abc"), copy1(8, 3), lit(b"!!"), copy2(5, 13)),
     b"abc" + b"abcabcab" + b"!!" + b"abcab"),
]

INVALID = [
    ("copy_offset_zero", stream(5, lit(b"a"), copy1(4, 0))),  # 2.2: offset 0 is not legal
    ("copy_past_output", stream(5, lit(b"a"), copy1(4, 2))),  # offset > decompressed position
    ("starts_with_copy", stream(4, copy1(4, 1))),  # "cannot start with a copy"
    ("length_longer_than_data", stream(10, lit(b"abc"))),
    ("length_shorter_than_data", stream(2, lit(b"abc"))),
    ("truncated_literal", stream(10, bytes([9 << 2]) + b"abc")),
    ("truncated_copy", stream(8, lit(b"abcd"), bytes([0x02 | (3 << 2), 0x04]))),
]


def test_preamble_examples_of_the_description():
    # format_description.txt:23-25
    assert varint(64) == b"\x40"
    assert varint(2097150) == b"\xFE\xFF\x7F"


@pytest.mark.parametrize("name,comp,raw", VALID, ids=[v[0] for v in VALID])
def test_host_decoder_known_answers(name, comp, raw):
    from brpc_amd import native
    assert native.snappy_uncompress(comp) == raw


@pytest.mark.parametrize("name,comp", INVALID, ids=[v[0] for v in INVALID])
def test_host_decoder_rejects_illegal_streams(name, comp):
    from brpc_amd import native
    with pytest.raises(ValueError):
        native.snappy_uncompress(comp)


def test_host_decoder_2097150_byte_preamble_example():
    # the description's 2 MiB length, reached with 2-byte-offset RLE copies
    n = 2097150
    elems = [lit(b"0123456789abcdef")]
    left = n - 16
    while left:
        k = min(64, left)
        elems.append(copy2(k, 16))
        left -= k
    comp = stream(n, *elems)
    assert comp[:3] == b"\xFE\xFF\x7F"
    from brpc_amd import native
    assert native.snappy_uncompress(comp) == (b"0123456789abcdef" * (n // 16 + 1))[:n]


def test_host_compressor_output_is_read_back_by_the_spec_reader():
    """Our compressor's output decoded by a from-the-description python
    reader (independent of the C++ decoder)."""
    from brpc_amd import native

    def spec_reader(s):
        pos, ulen, shift = 0, 0, 0
        while True:
            b = s[pos]
            pos += 1
            ulen |= (b & 0x7F) << shift
            shift += 7
            if not b & 0x80:
                break
        out = bytearray()
        while pos < len(s):
            tag = s[pos]
            pos += 1
            kind = tag & 3
            if kind == 0:
                n = tag >> 2
                if n >= 60:
                    k = n - 59
                    n = int.from_bytes(s[pos:pos + k], "little")
                    pos += k
                n += 1
                out += s[pos:pos + n]
                pos += n
                continue
            if kind == 1:
                length = ((tag >> 2) & 7) + 4
                off = ((tag >> 5) << 8) | s[pos]
                pos += 1
            else:
                length = (tag >> 2) + 1
                k = 2 if kind == 2 else 4
                off = int.from_bytes(s[pos:pos + k], "little")
                pos += k
            assert 0 < off <= len(out)
            for _ in range(length):
                out.append(out[-off])
        assert len(out) == ulen
        return bytes(out)

    text = b"".join(b"rpc %d channel server fiber xgmi " % (i % 97) for i in range(5000))
    for data in (b"", b"a", text, bytes(range(256)) * 300):
        assert spec_reader(native.snappy_compress(data)) == data


@pytest.mark.gpu
def test_gpu_decoder_known_answers_in_one_launch():
    torch = pytest.importorskip("torch")
    from brpc_amd.ops import snappy_decompress
    comps = [c for _, c, _ in VALID]
    raws = [r for _, _, r in VALID]
    packed = b"".join(comps)
    offs, pos = [], 0
    for c in comps:
        offs.append(pos)
        pos += len(c)
    d = torch.frombuffer(bytearray(packed), dtype=torch.uint8).to("cuda:0")
    out = snappy_decompress(d, offs, [len(c) for c in comps], [len(r) for r in raws])
    assert bytes(out.cpu().numpy().tobytes()) == b"".join(raws)


@pytest.mark.gpu
@pytest.mark.parametrize("name,comp", INVALID, ids=[v[0] for v in INVALID])
def test_gpu_decoder_rejects_illegal_streams(name, comp):
    torch = pytest.importorskip("torch")
    from brpc_amd.ops import snappy_decompress
    # the declared length (from the preamble) is what the caller passes
    ulen, shift, pos = 0, 0, 0
    while True:
        b = comp[pos]
        pos += 1
        ulen |= (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            break
    d = torch.frombuffer(bytearray(comp), dtype=torch.uint8).to("cuda:0")
    with pytest.raises(ValueError):
        snappy_decompress(d, [0], [len(comp)], [max(ulen, 1)])


@pytest.mark.gpu
def test_gpu_device_split_known_answers_and_rejects():
    """The same vectors through the device splitter + piece decoder (whole
    streams, no host tag walk). The 2 MiB preamble example is one unbroken
    chain of offset-16 copies: no 64 KiB fragment boundary can cut it, so
    the device refuses it (the RPC codec then decodes on the CPU)."""
    torch = pytest.importorskip("torch")
    from brpc_amd.ops import snappy_decompress_streams
    n = 2097150
    big = [lit(b"0123456789abcdef")]
    left = n - 16
    while left:
        k = min(64, left)
        big.append(copy2(k, 16))
        left -= k
    comps = [c for _, c, _ in VALID]
    raws = [r for _, _, r in VALID]
    packed = b"".join(comps)
    offs, pos = [], 0
    for c in comps:
        offs.append(pos)
        pos += len(c)
    d = torch.frombuffer(bytearray(packed), dtype=torch.uint8).to("cuda:0")
    out = snappy_decompress_streams(d, offs, [len(c) for c in comps], [len(r) for r in raws])
    assert bytes(out.cpu().numpy().tobytes()) == b"".join(raws)
    chain = stream(n, *big)
    d = torch.frombuffer(bytearray(chain), dtype=torch.uint8).to("cuda:0")
    with pytest.raises(ValueError):
        snappy_decompress_streams(d, [0], [len(chain)], [n])
    for name, comp in INVALID:
        ulen, shift, pos = 0, 0, 0
        while True:
            b = comp[pos]
            pos += 1
            ulen |= (b & 0x7F) << shift
            shift += 7
            if not b & 0x80:
                break
        d = torch.frombuffer(bytearray(comp), dtype=torch.uint8).to("cuda:0")
        with pytest.raises(ValueError):
            snappy_decompress_streams(d, [0], [len(comp)], [max(ulen, 1)])
