"""GPU JSON structural index (gpu/json_kernels.hip) against the pure-python
reference walk of the same bytes: real json.dumps documents (escapes,
unicode, nesting), adversarial backslash/quote soups whose runs straddle
64-byte lane and 16 KiB tile boundaries, inputs past 4096 tiles (the tile
scan carries state and offsets across LDS chunks), unaligned views and the
error codes."""
import json
import os
import random

import pytest

torch = pytest.importorskip("torch")

from brpc_amd.ops.json import json_index_host  # noqa: E402


@pytest.fixture(scope="module")
def dev():
    from brpc_amd import native
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    assert native.gpu.device_count() > 0
    return torch.device("cuda", 0)


def _doc(rnd, depth=0):
    k = rnd.random()
    if depth > 4 or k < 0.3:
        return rnd.choice([
            rnd.randint(-10**12, 10**12), rnd.random(), True, None,
            "".join(rnd.choice('ab"\\/\n\t{}[]:,é中') for _ in range(rnd.randint(0, 20))),
        ])
    if k < 0.65:
        return [_doc(rnd, depth + 1) for _ in range(rnd.randint(0, 6))]
    return {"k%d\"{" % i: _doc(rnd, depth + 1) for i in range(rnd.randint(0, 6))}


def _run(dev, data):
    from brpc_amd.ops import json_index
    buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev) if data else torch.empty(0, dtype=torch.uint8,
                                                                                                   device=dev)
    return json_index(buf).cpu().tolist()


def test_host_reference_matches_json_structure():
    # CPU: the reference walk agrees with the structure json.dumps wrote
    rnd = random.Random(3)
    for _ in range(50):
        obj = _doc(rnd)
        text = json.dumps(obj, ensure_ascii=rnd.random() < 0.5).encode()
        pos, open_ = json_index_host(text)
        assert not open_
        toks = bytes(text[p] for p in pos)
        assert toks.count(b'"'[0]) % 2 == 0
        assert toks.count(b"{"[0]) == toks.count(b"}"[0]) and toks.count(b"["[0]) == toks.count(b"]"[0])
    assert json_index_host(b'{"a\\"b": [1, "x,y"]}') == ([0, 1, 6, 7, 9, 11, 13, 17, 18, 19], False)
    assert json_index_host(b'"abc')[1]


@pytest.mark.gpu
def test_json_documents(dev):
    rnd = random.Random(11)
    for _ in range(40):
        text = json.dumps([_doc(rnd) for _ in range(rnd.randint(1, 40))], ensure_ascii=rnd.random() < 0.5).encode()
        assert _run(dev, text) == json_index_host(text)[0]


@pytest.mark.gpu
@pytest.mark.parametrize("alphabet", ['"\\a', '"\\\\\\a{', '"\\{}[]:,xy '])
def test_adversarial_escapes(dev, alphabet):
    # soups of quotes and backslash runs: every lane and tile boundary sees
    # odd and even runs and open strings; the stream closes its last string
    rnd = random.Random(hash(alphabet) & 0xFFFF)
    for n in (1, 63, 64, 65, 4095, 16383, 16384, 16385, 70000):
        s = "".join(rnd.choice(alphabet) for _ in range(n)).encode()
        pos, open_ = json_index_host(s)
        if open_:
            s += b'"'
            pos, open_ = json_index_host(s)
            if open_:  # the added quote was escaped
                s += b' "'
                pos, open_ = json_index_host(s)
        assert not open_
        assert _run(dev, s) == pos, n


@pytest.mark.gpu
def test_backslash_lanes_and_tiles(dev):
    # whole lanes (and a whole tile) of backslashes inside a string, both parities
    for run in (63, 64, 65, 127, 128, 129, 16384, 16385):
        for lead in (0, 1, 30, 62, 63):
            s = b" " * lead + b'["' + b"\\" * run + b'x", "y"]'
            pos, open_ = json_index_host(s)
            if open_:
                s += b'"]'
                pos, open_ = json_index_host(s)
            assert not open_
            assert _run(dev, s) == pos, (run, lead)


@pytest.mark.gpu
def test_many_tiles(dev):
    # > 4096 tiles: the tile scan carries state and offsets across LDS chunks. The input
    # repeats an odd-length unit, so the expected index is the unit's index
    # shifted by k * len(unit)
    rnd = random.Random(5)
    unit = (json.dumps({"a\\\\\"": [_doc(rnd) for _ in range(8)], "s": "x\\\"y"}) + ",").encode()
    if len(unit) % 2 == 0:
        unit = b" " + unit
    reps = (70 << 20) // len(unit) + 1
    upos = torch.tensor(json_index_host(unit)[0], dtype=torch.int64)
    expect = (upos[None, :] + torch.arange(reps, dtype=torch.int64)[:, None] * len(unit)).reshape(-1)
    from brpc_amd.ops import json_index
    buf = torch.frombuffer(bytearray(unit * reps), dtype=torch.uint8).to(dev)
    got = json_index(buf).cpu()
    assert got.numel() == expect.numel()
    assert torch.equal(got, expect)


@pytest.mark.gpu
def test_unaligned_view_and_errors(dev):
    from brpc_amd.ops import json_index
    text = json.dumps({"k": ["v\\\"", 1, {"z": [2, 3]}]}).encode() * 300
    big = torch.frombuffer(bytearray(b"xyz" + text), dtype=torch.uint8).to(dev)
    assert json_index(big[3:]).cpu().tolist() == json_index_host(text)[0]
    assert _run(dev, b"") == []
    with pytest.raises(ValueError, match="unterminated"):
        _run(dev, b'{"a": "b')
    with pytest.raises(ValueError, match="structural positions"):
        json_index(torch.frombuffer(bytearray(b"[1,2,3,4]"), dtype=torch.uint8).to(dev), max_positions=3)
    with pytest.raises(ValueError):
        json_index(torch.zeros(4, dtype=torch.uint8))


def _echo_doc(n):
    # an example.EchoRequest as JSON whose message is long and escape-heavy
    body = ("plain text run " * 40 + 'q"uote \\ back\\slash é 中 ') * n
    return json.dumps({"message": body, "sleep_us": 7, "server_fail": False}).encode(), body


def test_json2pb_round_trip_cpu():
    from brpc_amd import native
    text, body = _echo_doc(3)
    out = json.loads(native.json_to_pb_to_json("example.EchoRequest", text))
    assert out["message"] == body and out["sleep_us"] == 7
    with pytest.raises(RuntimeError):
        native.json_to_pb_to_json("example.EchoRequest", text[:-5])


@pytest.mark.gpu
@pytest.mark.parametrize("direct", [True, False])
def test_json_index_bytes_matches_host(dev, direct):
    """Through the offload entry: pinned in/out read and written by the
    kernel directly, or staged through HBM."""
    from brpc_amd import native
    native.set_flag("json_index_direct_host", "true" if direct else "false")
    try:
        rnd = random.Random(9)
        text = json.dumps([_doc(rnd) for _ in range(300)]).encode()
        assert native.gpu.json_index_bytes(text, 0) == json_index_host(text)[0]
        for k in (1, 63, 64, 65, 4097):  # prefixes: tails in every lane position, some inside a string
            want, still_open = json_index_host(text[:k])
            if still_open:
                with pytest.raises(RuntimeError):
                    native.gpu.json_index_bytes(text[:k], 0)
            else:
                assert native.gpu.json_index_bytes(text[:k], 0) == want
        with pytest.raises(RuntimeError):
            native.gpu.json_index_bytes(b'{"open', 0)
    finally:
        native.set_flag("json_index_direct_host", "true")


@pytest.mark.gpu
def test_json2pb_uses_device_index_for_large_bodies(dev):
    """json2pb with the device index installed: bodies at or above the
    threshold are indexed on the GPU (stats move) and parse to exactly what
    the CPU-only parser produces; smaller bodies stay on the CPU."""
    from brpc_amd import native
    text, body = _echo_doc(400)  # ~400 KiB
    small, _ = _echo_doc(1)
    cpu_big = native.json_to_pb_to_json("example.EchoRequest", text)
    native.gpu.enable_json_index(0, 65536)
    native.set_flag("json_index_min_density", "0")  # this one long string would be left to the host
    try:
        s0 = native.gpu.json_stats()
        assert native.json_to_pb_to_json("example.EchoRequest", text) == cpu_big
        s1 = native.gpu.json_stats()
        assert s1["indexed_bodies"] == s0["indexed_bodies"] + 1 and s1["indexed_bytes"] - s0["indexed_bytes"] == len(text)
        assert json.loads(cpu_big)["message"] == body
        native.json_to_pb_to_json("example.EchoRequest", small)
        assert native.gpu.json_stats()["indexed_bodies"] == s1["indexed_bodies"]
        # malformed large body (cut inside the message string): the device
        # reports the open string, the CPU parser reports the error
        with pytest.raises(RuntimeError):
            native.json_to_pb_to_json("example.EchoRequest", text[:100000])
        assert native.gpu.json_stats()["failures"] == s1["failures"] + 1
    finally:
        native.set_flag("json_index_min_density", "8")
        native.gpu.disable_json_index()


@pytest.mark.gpu
def test_structurally_sparse_bodies_stay_on_the_host(dev):
    """A body that is mostly one long string has too few structural
    characters for the device index to pay (-json_index_min_density): it is
    parsed by the host parser, with the same result; a dense body of the
    same size is indexed."""
    from brpc_amd import native
    sparse = json.dumps({"message": "x" * 200000, "sleep_us": 1}).encode()
    dense = json.dumps({"message": "m", "ids": list(range(40000))}).encode()
    native.gpu.enable_json_index(0, 65536)
    try:
        s0 = native.gpu.json_stats()
        out = native.json_to_pb_to_json("example.EchoRequest", sparse)
        s1 = native.gpu.json_stats()
        assert json.loads(out)["message"] == "x" * 200000
        assert s1["sparse_skips"] == s0["sparse_skips"] + 1
        assert s1["indexed_bodies"] == s0["indexed_bodies"]
        out = native.json_to_pb_to_json("example.EchoRequest", dense)
        s2 = native.gpu.json_stats()
        assert json.loads(out)["ids"] == list(range(40000))
        assert s2["indexed_bodies"] == s1["indexed_bodies"] + 1
    finally:
        native.gpu.disable_json_index()


def _jsonout_fixture(tmp_path):
    """The reference's test/jsonout document and its schema (message.proto),
    shipped with the tests as tests/fixtures/ref_jsonout.tar.gz so the GPU
    parity check runs wherever the tests do (the reference tree is not on
    the GPU box). Returns (directory, document bytes)."""
    import tarfile
    with tarfile.open(os.path.join(os.path.dirname(__file__), "fixtures", "ref_jsonout.tar.gz")) as t:
        for name in ("jsonout", "message.proto"):
            m = t.getmember(name)
            assert m.isfile()
            with open(os.path.join(tmp_path, name), "wb") as f:
                f.write(t.extractfile(m).read())
    with open(os.path.join(tmp_path, "jsonout"), "rb") as f:
        return str(tmp_path), f.read()


@pytest.mark.gpu
def test_reference_jsonout_fixture_through_device_index(dev, tmp_path):
    """The reference's 98 KB test/jsonout document (gss_us_res_t) parsed with
    the GPU structural index gives exactly the CPU parser's message."""
    from brpc_amd import native
    ref, text = _jsonout_fixture(tmp_path)
    cpu = native.json_proto_roundtrip(ref, "message.proto", "gss.message.gss_us_res_t", text, False)
    native.gpu.enable_json_index(0, 4096)
    try:
        s0 = native.gpu.json_stats()
        gpu = native.json_proto_roundtrip(ref, "message.proto", "gss.message.gss_us_res_t", text, False)
        s1 = native.gpu.json_stats()
    finally:
        native.gpu.disable_json_index()
    assert s1["indexed_bodies"] == s0["indexed_bodies"] + 1
    assert gpu == cpu
    assert json.loads(gpu[0]) == json.loads(text)
