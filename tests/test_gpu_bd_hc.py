"""GPU parity for block-dependent frames at compression level >= 3, SURVEY.md §8(f).

The reference's compressBlockDependency (src/lz4mt.cpp:460-538) with
isHc = level >= 3 drives lz4 1.9.3's legacy HC stream
(src/lz4mt.cpp:295-332): LZ4_resetStreamStateHC (level 9 whatever the level
asked), LZ4_compressHC_limitedOutput_continue per block (cap = inSize - 1),
LZ4_slideInputBufferHC (a reset) when the next block would not fit the
input buffer.  Golden frames: that sequence replayed on liblz4
(tests/golden/make_golden.py: bd_hc_frame_reference); larger inputs: the
oracle's restatement (oracle.bd_hc_frame, pinned to the golden frames by
tests/test_oracle.py).
"""
import pytest
import torch
import xxhash

import oracle
from conftest import bd_data, bd_input, read_golden

pytestmark = pytest.mark.gpu

L = None


@pytest.fixture(scope="module", autouse=True)
def lib():
    global L
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    import lz4mt_amd
    L = lz4mt_amd
    return L


def dev(b):
    t = torch.empty(max(len(b), 1), dtype=torch.uint8, device="cuda")
    if b:
        t[:len(b)].copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
    return t[:len(b)]


def host(t):
    return bytes(t.cpu().numpy().tobytes())


def _sd(f):
    return L.make_sd(f["bid"], f["stream_checksum"], f["block_checksum"], block_dependence=True)


@pytest.mark.parametrize("level", [3, 9, 12])
def test_bd_hc_golden_frames_device(golden, level):
    """Every level >= 3 gives the same frame: the HC stream runs at level 9."""
    for f in golden["bd_hc_frames"]:
        data = bd_data(f)
        frame = read_golden(f["file"])
        got = host(L.compress_frame(dev(data), _sd(f), level=level))
        assert got == frame, (f["name"], level)
        out, r = L.decompress_frame(dev(frame))
        assert r == 0 and host(out) == data, f["name"]


def test_bd_hc_known_answers_device(golden):
    for f in golden["bd_hc_known"]:
        data = bd_input(f["bytes"], f["seed"])
        frame = L.compress_frame(dev(data), _sd(f), level=9)
        assert (frame.numel(), L.xxh32(frame)) == (f["size"], f["xxh32"]), f["name"]
        out, r = L.decompress_frame(frame)
        assert r == 0 and L.xxh32(out) == f["content_xxh32"], f["name"]


@pytest.mark.parametrize("mode", ["DEVICE", "PARALLEL"])
@pytest.mark.parametrize("batches", ["one", "many"])
def test_bd_hc_callback_api(golden, monkeypatch, mode, batches):
    """lz4mtCompress at level 9 on -BD frames; with 1 MiB batches a 64 KiB
    block's segment (17 blocks, 1088 KiB) starts in the batch before, so its
    chain and matches reach into the carried 64 KiB history."""
    if batches == "many":
        monkeypatch.setenv("LZ4MT_AMD_BATCH0_MIB", "1")
        monkeypatch.setenv("LZ4MT_AMD_BATCH_MIB", "1")
    m = {"DEVICE": L.MODE_DEVICE, "PARALLEL": L.MODE_PARALLEL}[mode]
    for f in golden["bd_hc_frames"] + golden["bd_hc_known"]:
        data = bd_data(f) if "file" in f else bd_input(f["bytes"], f["seed"])
        r, frame = L.compress(data, _sd(f), mode=m, level=9)
        assert r == 0, (f["name"], L.result_to_string(r))
        if "file" in f:
            assert frame == read_golden(f["file"]), (f["name"], mode, batches)
        else:
            assert (len(frame), xxhash.xxh32(frame).intdigest()) == (f["size"], f["xxh32"]), (f["name"], mode)
        r, out, sd = L.decompress(frame, len(data) + 64, mode=m)
        assert r == 0 and out == data, (f["name"], mode, batches, L.result_to_string(r))


@pytest.mark.parametrize("bid,kind", [(4, "bd"), (5, "mixed"), (6, "bd"), (7, "zeros"), (4, "random")])
def test_bd_hc_vs_oracle_48mib(bid, kind):
    """48 MiB + a ragged tail against the oracle's HC stream, byte for byte."""
    f = {"bytes": (48 << 20) + 12345, "seed": 70 + bid, "kind": kind}
    data = bd_data(f)
    want = oracle.bd_hc_frame(data, bid, True, True)
    sd = L.make_sd(bid, True, True, block_dependence=True)
    got = L.compress_frame(dev(data), sd, level=9)
    assert (got.numel(), L.xxh32(got)) == (len(want), xxhash.xxh32(want).intdigest()), (bid, kind)
    out, r = L.decompress_frame(got)
    assert r == 0 and L.xxh32(out) == xxhash.xxh32(data).intdigest()
