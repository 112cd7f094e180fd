"""GPU parity for LZ4-HC (compression levels 3..12), SURVEY.md §8(f) #3.

The reference selects LZ4_compressHC2_limitedOutput(src, dst, n, cap = n,
level) for ctx.compressionLevel >= 3 (src/main.cpp:778-785) and stores a
block raw when it returns <= 0 (src/lz4mt.cpp:391-394).  The GPU encoder
(lz4mt_hc.hip) must produce the same bytes: against liblz4 1.9.3's own
outputs (tests/golden/golden.json "hc_blocks", made by make_golden.py) and
against the oracle's restatement (oracle/lz4hc_oracle.c, pinned against
liblz4 by tests/test_oracle.py).
"""
import hashlib
import random
import struct

import pytest
import torch
import xxhash

import oracle
from conftest import bd_input

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


def hc_frame(data, bid, sck, bck, level):
    """lz4mt frame of HC blocks (src/lz4mt.cpp:372-457 with the HC codec), from the oracle."""
    head = oracle.compress_frame(b"", oracle.params(bid, sck, bck))[:7]
    out = bytearray(head)
    bm = 1 << (8 + 2 * bid)
    for off in range(0, len(data), bm):
        p = data[off:off + bm]
        c = oracle.compress_block_hc(p, len(p), level)
        stored = c if c else p
        out += struct.pack("<I", len(c) if c else len(p) | 0x80000000) + stored
        if bck:
            out += struct.pack("<I", xxhash.xxh32(stored).intdigest())
    out += b"\0\0\0\0"
    if sck:
        out += struct.pack("<I", xxhash.xxh32(data).intdigest())
    return bytes(out)


def test_hc_blocks_golden(golden, golden_inputs):
    inputs = dict(golden_inputs)
    inputs["bdmix300k"] = bd_input(300_000, 31)
    for v in golden["hc_blocks"]:
        data = inputs[v["input"]][:v["n"]]
        c = L.compress_block(data, v["cap"], level=v["level"])
        assert len(c) == v["ret"] and hashlib.sha1(c).hexdigest() == v["sha1"], v


def _mixed(n, seed):
    rnd = random.Random(seed)
    syn = oracle.gen_synthetic(1 << 20, seed)
    out = bytearray()
    while len(out) < n:
        k = rnd.randrange(6)
        if k == 0:
            a = rnd.randrange(len(syn) - 5000)
            out += syn[a:a + rnd.randrange(50, 5000)]
        elif k == 1:
            out += bytes([rnd.randrange(256)]) * rnd.randrange(1, 3000)
        elif k == 2 and len(out) > 10:
            a = rnd.randrange(max(0, len(out) - 70000), len(out))
            out += out[a:a + rnd.randrange(4, 3000)]
        elif k == 3:
            out += oracle.gen_random(rnd.randrange(10, 500), rnd.randrange(1 << 30))
        elif k == 4:
            p = bytes(rnd.randrange(256) for _ in range(rnd.randrange(2, 9)))
            out += p * rnd.randrange(2, 300)
        else:
            out += b"\0" * rnd.randrange(1, 70000)
    return bytes(out[:n])


def test_hc_blocks_fuzz_vs_oracle():
    for seed in range(16):
        rnd = random.Random(seed)
        d = _mixed(rnd.choice([13, 14, 100, 5000, 65547, 300_000, 1 << 20]), seed)
        for level in (3, rnd.choice([4, 5, 6, 7, 8]), 9):
            for cap in (len(d), len(d) - 1, len(d) // 3):
                assert L.compress_block(d, cap, level=level) == oracle.compress_block_hc(d, cap, level), \
                    (seed, len(d), level, cap)


def test_hc_opt_blocks_fuzz_vs_oracle():
    """Levels 10..12 (LZ4HC_compress_optimal: price table, chain swap, full
    update at 12) and 17 (the reference CLI's -A, clamped to 12)."""
    for seed in range(10):
        rnd = random.Random(100 + seed)
        d = _mixed(rnd.choice([12, 13, 14, 100, 5000, 65547, 200_000]), 100 + seed)
        for level in (10, 11, 12, 17):
            for cap in (len(d), len(d) - 1, len(d) // 3):
                assert L.compress_block(d, cap, level=level) == oracle.compress_block_hc(d, cap, level), \
                    (seed, len(d), level, cap)
    for d in (oracle.gen_synthetic(300_000, 5), bytes(100_000), oracle.gen_random(70_000, 4)):
        for level in (10, 12):
            assert L.compress_block(d, len(d), level=level) == oracle.compress_block_hc(d, len(d), level), level


@pytest.mark.parametrize("bid,sck,bck,level", [(4, True, True, 9), (5, False, True, 3), (7, True, False, 9),
                                               (6, False, False, 6), (5, True, True, 12), (6, False, True, 10),
                                               (5, False, True, 17), (7, True, True, 12)])
def test_hc_frames_device(bid, sck, bck, level):
    data = oracle.gen_synthetic(3 << 20, 7) + bd_input(2 << 20, 8) + bytes(300_000) + oracle.gen_random(70_000, 2)
    want = hc_frame(data, bid, sck, bck, level)
    fr = L.compress_frame(dev(data), L.make_sd(bid, sck, bck), level=level)
    assert host(fr) == want
    out, r = L.decompress_frame(fr)
    assert r == 0 and host(out) == data


@pytest.mark.parametrize("mode", ["DEVICE", "SEQUENTIAL"])
def test_hc_opt_callback_api(mode):
    """lz4mtCompress at ctx.compressionLevel = 12 (the optimal parser) through
    the batch engine and through the GPU block operator per block."""
    m = {"DEVICE": L.MODE_DEVICE, "SEQUENTIAL": L.MODE_SEQUENTIAL}[mode]
    data = oracle.gen_synthetic(600_000, 19) + bd_input(300_000, 20)
    r, frame = L.compress(data, L.make_sd(5, True, True), mode=m, level=12)
    assert r == 0, L.result_to_string(r)
    assert frame == hc_frame(data, 5, True, True, 12), mode
    r, out, _ = L.decompress(frame, len(data) + 64, mode=m)
    assert r == 0 and out == data


@pytest.mark.parametrize("mode", ["DEVICE", "PARALLEL", "SEQUENTIAL"])
def test_hc_callback_api(mode):
    """lz4mtCompress with ctx.compressionLevel = 9 and null codecs: the batch
    engine (DEVICE, PARALLEL) or the GPU block operator per block
    (SEQUENTIAL) -- the reference's frame with HC blocks either way."""
    m = {"DEVICE": L.MODE_DEVICE, "PARALLEL": L.MODE_PARALLEL, "SEQUENTIAL": L.MODE_SEQUENTIAL}[mode]
    data = oracle.gen_synthetic(1 << 20, 9) + bd_input(600_000, 10)
    for bid, sck, bck in ((4, True, True), (6, False, True)):
        r, frame = L.compress(data, L.make_sd(bid, sck, bck), mode=m, level=9)
        assert r == 0, L.result_to_string(r)
        assert frame == hc_frame(data, bid, sck, bck, 9), (mode, bid)
        r, out, _ = L.decompress(frame, len(data) + 64, mode=m)
        assert r == 0 and out == data


def test_hc_256mib_properties():
    """App. F 256 MiB at level 9, 4 MiB blocks: round trip, and the first
    and last block against the oracle."""
    n = 256 << 20
    src = L.gen_synthetic(n, seed=42)
    fr = L.compress_frame(src, L.make_sd(7, False, True), level=9)
    out, r = L.decompress_frame(fr)
    assert r == 0 and out.numel() == n and L.xxh32(out) == 0xE6F24EBA
    hl, recs, _ = L.frame_records(fr)
    for b in (0, len(recs) - 2):
        blk = host(src[b * (4 << 20):(b + 1) * (4 << 20)])
        want = oracle.compress_block_hc(blk, len(blk), 9)
        size = int.from_bytes(host(fr[recs[b]:recs[b] + 4]), "little")
        assert size == len(want) and host(fr[recs[b] + 4:recs[b] + 4 + size]) == want, b
    assert fr.numel() < 0.45 * n   # HC-9 compresses App. F input well below the fast parser's 1/2.025


def _split_input(kind, n, seed):
    if kind == "appf":
        return oracle.gen_synthetic(n, seed)
    if kind == "mixed":
        return _mixed(n, seed)
    if kind == "runs":   # long zero runs across the streams' starts, random between
        rnd = random.Random(seed)
        out = bytearray()
        while len(out) < n:
            out += bytes(rnd.randrange(100_000, 900_000)) + oracle.gen_random(rnd.randrange(10, 90_000), seed)
        return bytes(out[:n])
    if kind == "random":
        return oracle.gen_random(n, seed)
    return bd_input(n, seed)


@pytest.mark.parametrize("sub", ["64", "256", "0"])
@pytest.mark.parametrize("kind", ["appf", "mixed", "runs", "bd", "random"])
def test_hc_split_parse_vs_oracle(monkeypatch, sub, kind):
    """Blocks of >= 2 streams are parsed by one wave per stream and spliced
    where the parses meet (lz4mt_hc.hip k_hc_heads / k_hc_exit / k_hc_join;
    blocks that do not meet are re-run whole): the same bytes as the serial
    parse at every stream length (LZ4MT_AMD_HC_SUB_KIB; 0 = no split)."""
    monkeypatch.setenv("LZ4MT_AMD_HC_SUB_KIB", sub)
    data = _split_input(kind, (9 << 20) + 4321, 3)
    for bid, level in ((7, 9), (6, 5)):
        want = hc_frame(data, bid, False, True, level)
        fr = L.compress_frame(dev(data), L.make_sd(bid, False, True), level=level)
        assert host(fr) == want, (sub, kind, bid, level)
    out, r = L.decompress_frame(fr)
    assert r == 0 and host(out) == data


@pytest.mark.parametrize("sub", ["64", "256", "0"])
@pytest.mark.parametrize("kind", ["appf", "mixed", "runs", "random"])
def test_hc_opt_split_parse_vs_oracle(monkeypatch, sub, kind):
    """The optimal parser (levels >= 10) on the split path: one wave and one
    price table per stream, spliced where the parses meet at a loop top
    with anchor == ip (k_hc_opt_heads / k_hc_opt_exit / k_hc_join)."""
    monkeypatch.setenv("LZ4MT_AMD_HC_SUB_KIB", sub)
    data = _split_input(kind, (5 << 20) + 4321, 5)
    for bid, level in ((7, 12), (6, 10)):
        want = hc_frame(data, bid, False, True, level)
        fr = L.compress_frame(dev(data), L.make_sd(bid, False, True), level=level)
        assert host(fr) == want, (sub, kind, bid, level)
    out, r = L.decompress_frame(fr)
    assert r == 0 and host(out) == data
    d = data[:(1 << 20) + 12345]
    for cap in (len(d), len(d) - 1):
        assert L.compress_block(d, cap, level=11) == oracle.compress_block_hc(d, cap, 11), (sub, kind, cap)


@pytest.mark.parametrize("kind", ["appf", "mixed", "random"])
def test_hc_block_operator_split(kind):
    """lz4mtHipCompressBlock on 1-4 MiB blocks runs the split parse too
    (one wave per 256 KiB stream): the oracle's bytes at caps n, n - 1, a
    tight cap and a cap past the bound."""
    rnd = random.Random(len(kind))
    for n in (4 << 20, (1 << 20) + 12345):
        d = _split_input(kind, n, rnd.randrange(1000))
        want_n = oracle.compress_block_hc(d, n, 9)
        for cap in (n, n - 1, max(len(want_n), 1) - 1 if want_n else n // 2, n + n // 255 + 16):
            assert L.compress_block(d, cap, level=9) == oracle.compress_block_hc(d, cap, 9), (kind, n, cap)
