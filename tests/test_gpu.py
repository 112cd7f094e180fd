"""GPU parity tests: the HIP path (through the C ABI) against the oracle and
the golden fixtures.  Bit-exact everywhere: this path is byte/integer work.

Sizes: golden fixtures (bytes .. 300 KB), random block fuzz vs the oracle,
the SURVEY.md App. F known answers at 256 MiB (frame size + XXH32 for all 10
flag rows), and a 2 GiB round trip checked through size-independent
properties (XXH32 of input == XXH32 of output, per-block checksums verified
by the decoder, block sample vs the oracle).
"""
import ctypes
import os
import random

import pytest
import torch
import xxhash

import oracle
from conftest import read_golden, with_stream_size

pytestmark = pytest.mark.gpu

L = None


@pytest.fixture(scope="module", autouse=True)
def lib():
    global L
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    import lz4mt_amd
    L = lz4mt_amd
    assert L.device_count() > 0
    return L


def dev(b):
    t = torch.empty(max(len(b), 1), dtype=torch.uint8, device="cuda")
    if b:
        t[:len(b)].copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
    return t[:len(b)]


def host(t):
    return bytes(t.cpu().numpy().tobytes())


def test_p17_and_base_encoders_agree(monkeypatch):
    """k_encode_p17 (the 3-byte table; the default at 256 KiB blocks) and
    k_encode (the default above) forced either way write the same frames,
    byte for byte (B5 and B6)."""
    src = L.gen_synthetic(12 << 20, seed=5, device="cuda")
    for bid in (5, 6):
        sd = L.make_sd(bid, stream_checksum=False, block_checksum=True)
        want = host(L.compress_frame(src, sd))
        for enc in ("p17", "base"):
            monkeypatch.setenv("LZ4MT_AMD_ENC", enc)
            got = host(L.compress_frame(src, sd))
            monkeypatch.delenv("LZ4MT_AMD_ENC")
            assert got == want, (bid, enc)
    data = host(src[:(3 << 20) + 12345])
    sd = L.make_sd(5, stream_checksum=True, block_checksum=True)
    assert host(L.compress_frame(dev(data), sd)) == oracle.compress_frame(data, oracle.params(5, True, True))


def test_encoder_lds_exchange_order():
    """The block encoder's table probe (LZ4MT_ENC_XCHG) takes each lane's
    candidate from one LDS exchange, which is LZ4's sequential insert order
    only if a wave's same-address exchanges apply in ascending lane order;
    the library checks that once per device before the first encode."""
    assert L.lib.lz4mtHipCheckEncoderOrder() == 1


# ---------------------------------------------------------------------------
# block operators (reference plugin signatures)
# ---------------------------------------------------------------------------
def test_block_compress_golden(golden, golden_inputs):
    import hashlib
    for v in golden["blocks"]:
        data = golden_inputs[v["input"]][:v["n"]]
        c = L.compress_block(data, v["cap"])
        assert len(c) == v["ret"] and hashlib.sha1(c).hexdigest() == v["sha1"], v


def test_block_compress_fuzz_vs_oracle():
    rnd = random.Random(3)
    syn = oracle.gen_synthetic(1 << 20)
    for t in range(80):
        n = rnd.choice([1, 7, 12, 13, 14, 20, 64, 100, 1000, 4095, 65535, 65546, 65547, 65548, 100_000, 262_144])
        kind = t % 5
        if kind == 0:
            d = syn[:n]
        elif kind == 1:
            d = bytes(rnd.randrange(3) for _ in range(n))
        elif kind == 2:
            d = oracle.gen_random(n, t)
        elif kind == 3:
            d = (bytes(rnd.randrange(256) for _ in range(rnd.randrange(1, 70))) * (n + 1))[:n]
        else:
            d = bytes(n)
        for cap in (n, max(n - 1, 0), n + n // 255 + 16, n // 2):
            assert L.compress_block(d, cap) == oracle.compress_block(d, cap), (t, n, cap)


def _mixed(n, seed):
    # synthetic text, random runs (long literal runs > 64), zero runs and
    # repeats (matches longer than one 256-byte count round), near/far offsets
    rnd = random.Random(seed)
    syn = oracle.gen_synthetic(1 << 20, seed)
    out, size = [], 0
    while size < n:
        k = rnd.randrange(5)
        if k == 0:
            a = rnd.randrange(len(syn) - 5000)
            piece = syn[a:a + rnd.randrange(100, 5000)]
        elif k == 1:
            piece = oracle.gen_random(rnd.randrange(65, 700), rnd.randrange(1 << 30))
        elif k == 2:
            piece = bytes(rnd.randrange(1, 3000))
        elif k == 3 and out:
            prev = b"".join(out[-8:])
            a = rnd.randrange(len(prev))
            piece = prev[a:a + rnd.randrange(4, 2000)]
        else:
            piece = bytes([rnd.randrange(256)]) * rnd.randrange(1, 400)
        out.append(piece)
        size += len(piece)
    return b"".join(out)[:n]


@pytest.mark.parametrize("n", [65547, 300_000, (4 << 20) - 1, 4 << 20, (4 << 20) + 1, 5 << 20])
def test_block_compress_mixed_vs_oracle(n):
    # both u32 encoder paths: tagged (n <= 4 MiB) and untagged (larger
    # blocks, reachable only through the block operator)
    d = _mixed(n, n)
    for cap in (n, n - 1, n + n // 255 + 16, n // 3):
        assert L.compress_block(d, cap) == oracle.compress_block(d, cap), (n, cap)


def test_block_decompress_golden(golden, decode_blob):
    for v in golden["decode"]:
        blk = decode_blob[v["off"]:v["off"] + v["len"]]
        r, out = L.decompress_block(blk, v["cap"])
        assert r == v["ret"], v
        if r >= 0:
            assert xxhash.xxh32(out).intdigest() == v["out_xxh32"], v


def test_block_decompress_crafted(golden):
    for v in golden["crafted"]:
        r, out = L.decompress_block(bytes.fromhex(v["block_hex"]), v["cap"])
        assert r == v["ret"], v
        if r >= 0:
            assert xxhash.xxh32(out).intdigest() == v["out_xxh32"], v


def test_block_decompress_long_matches():
    # long overlapping / far matches (ring and HBM paths of the decoder)
    rnd = random.Random(8)
    parts = []
    for i in range(300):
        parts.append(bytes([rnd.randrange(256)]) * rnd.randrange(1, 5000))
        parts.append(oracle.gen_random(rnd.randrange(1, 300), i))
    d = b"".join(parts)[:4 << 20]
    d = d + d[:40_000] + oracle.gen_synthetic(200_000)[:100_000] + d[100:70_000]
    for n in (len(d) // 3, len(d)):
        blk = oracle.compress_block(d[:n], n + n // 255 + 16)
        r, out = L.decompress_block(blk, 4 << 20 if n <= 4 << 20 else n)
        assert r == n and out == d[:n]


# ---------------------------------------------------------------------------
# device-resident frames
# ---------------------------------------------------------------------------
def test_gen_synthetic_matches_oracle():
    for n in (1, 65536, 100_000, 8 << 20):
        t = L.gen_synthetic(n)
        assert host(t) == oracle.gen_synthetic(n)
    assert L.xxh32(L.gen_synthetic(8 << 20)) == 0xD89F562C


def test_device_xxh32():
    rnd = random.Random(2)
    for n in (0, 1, 15, 16, 17, 1000, 65537):
        b = bytes(rnd.randrange(256) for _ in range(n))
        assert L.xxh32(dev(b)) == xxhash.xxh32(b).intdigest()


def test_frames_golden(golden, golden_inputs):
    for f in golden["frames"]:
        data = golden_inputs[f["input"]]
        sd = L.make_sd(f["bid"], f["stream_checksum"], f["block_checksum"])
        fr = L.compress_frame(dev(data), sd)
        assert host(fr) == read_golden(f["file"]), f["file"]
        out, r = L.decompress_frame(dev(read_golden(f["file"])))
        assert r == 0 and host(out) == data, f["file"]


def test_frame_decode_errors(golden_inputs):
    data = golden_inputs["syn300k"]
    f = host(L.compress_frame(dev(data), L.make_sd(5, True, True)))
    R = L.Result

    def code(b):
        out = torch.empty(len(data) + (1 << 20), dtype=torch.uint8, device="cuda")
        return L.decompress_frame(dev(b), out=out, check=False)[1]
    assert code(f) == R.OK
    assert code(b"\x01\x02\x03\x04rest") == R.INVALID_MAGIC_NUMBER
    bad = bytearray(f); bad[6] ^= 1
    assert code(bytes(bad)) == R.INVALID_HEADER_CHECKSUM
    bad = bytearray(f); bad[20] ^= 0xFF
    assert code(bytes(bad)) in (R.BLOCK_CHECKSUM_MISMATCH, R.DECOMPRESS_FAIL)
    assert code(f[:-2]) == R.CANNOT_READ_STREAM_CHECKSUM
    assert code(f[:100]) == R.CANNOT_READ_BLOCK_DATA
    bad = bytearray(f); bad[-1] ^= 1
    assert code(bytes(bad)) == R.STREAM_CHECKSUM_MISMATCH
    skip = (0x184D2A51).to_bytes(4, "little") + (5).to_bytes(4, "little") + b"12345"
    out = torch.empty(2 * len(data) + (1 << 20), dtype=torch.uint8, device="cuda")
    o, r = L.decompress_frame(dev(f + skip + f + b"junkjunk"), out=out, check=False)
    assert r == R.OK and host(o) == data + data


@pytest.fixture(scope="module")
def syn256():
    t = L.gen_synthetic(256 << 20)
    assert L.xxh32(t) == 0xE6F24EBA
    return t


@pytest.mark.parametrize("row", [
    ((1, 0, 7), 133159140, 0x157099A8), ((0, 0, 7), 133159136, 0x8AC5DBC8), ((1, 1, 7), 133159396, 0xC532D9D2),
    ((0, 1, 7), 133159392, 0x1686045A), ((1, 0, 4), 131940148, 0xFC3A55A1), ((1, 0, 5), 136141814, 0xAF5572EC),
    ((1, 0, 6), 133770948, 0x7D1BC1BA), ((0, 1, 4), 131956528, 0xAB492B3C), ((0, 1, 5), 136145906, 0xE62BB3AC),
    ((0, 1, 6), 133771968, 0x535404A3)])
def test_known_answers_256mib(row, syn256):
    (sc, bc, bid), size, h = row
    fr = L.compress_frame(syn256, L.make_sd(bid, bool(sc), bool(bc)))
    assert fr.numel() == size
    assert L.xxh32(fr) == h
    out, r = L.decompress_frame(fr)
    assert r == 0 and out.numel() == syn256.numel() and L.xxh32(out) == 0xE6F24EBA


def test_roundtrip_2gib_properties():
    n = 2 << 30
    src = L.gen_synthetic(n, seed=1234)
    h_in = L.xxh32(src)
    sd = L.make_sd(7, stream_checksum=False, block_checksum=True)
    fr = L.compress_frame(src, sd)
    # sample blocks against the oracle
    f_host_head = host(fr[:3 << 20])
    blk0 = oracle.compress_block(host(src[:4 << 20]), 4 << 20)
    assert f_host_head[7:11] == len(blk0).to_bytes(4, "little")
    assert f_host_head[11:11 + len(blk0)][:1 << 20] == blk0[:1 << 20]
    out, r = L.decompress_frame(fr)
    assert r == 0 and out.numel() == n
    assert L.xxh32(out) == h_in
    del out, fr, src
    torch.cuda.empty_cache()


def test_incompressible_is_raw():
    d = oracle.gen_random(3 << 20, 5)
    fr = host(L.compress_frame(dev(d), L.make_sd(6, True, True)))
    assert fr == oracle.compress_frame(d, oracle.params(6, True, True))
    assert int.from_bytes(fr[7:11], "little") == (1 << 20) | 0x80000000


# ---------------------------------------------------------------------------
# the lz4mt.h callback API on the GPU
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("mode", ["SEQUENTIAL", "PARALLEL", "DEVICE"])
def test_callback_api_on_gpu(golden_inputs, mode):
    m = {"SEQUENTIAL": L.MODE_SEQUENTIAL, "PARALLEL": L.MODE_PARALLEL, "DEVICE": L.MODE_DEVICE}[mode]
    data = golden_inputs["syn300k"] + golden_inputs["zeros300k"] + golden_inputs["random100k"]
    for bid, sck, bck in ((4, True, True), (7, True, False), (5, False, True)):
        sd = L.make_sd(bid, sck, bck)
        r, frame = L.compress(data, sd, mode=m)
        assert r == 0, L.result_to_string(r)
        assert frame == oracle.compress_frame(data, oracle.params(bid, sck, bck)), (mode, bid)
        r, out, _ = L.decompress(frame, len(data) + 64, mode=m)
        assert r == 0 and out == data, (mode, bid, L.result_to_string(r))


# ---------------------------------------------------------------------------
# the parallel frame walk (candidate offsets + pointer doubling) and the walk
# fused into the decode (k_decode_walk: records decoded as the walk publishes
# them) must give the serial walk's records, bytes and error codes on every
# frame, well-formed or not
# ---------------------------------------------------------------------------
def _decode_all(b, cap):
    res = []
    for mode in ("serial", "parallel", "fused"):
        os.environ["LZ4MT_AMD_WALK"] = mode
        try:
            out = torch.empty(cap, dtype=torch.uint8, device="cuda")
            o, r = L.decompress_frame(dev(b), out=out, check=False)
            res.append((r, host(o) if r == 0 else None))
        finally:
            del os.environ["LZ4MT_AMD_WALK"]
    return res


@pytest.mark.parametrize("bid,sck,bck", [(4, True, True), (4, False, False), (5, False, True), (6, False, True),
                                         (7, True, True), (7, False, False)])
def test_frame_walks_match_serial(golden_inputs, bid, sck, bck):
    data = (golden_inputs["syn300k"] + golden_inputs["zeros300k"] + golden_inputs["random100k"]) * 3
    if bid >= 6:   # several blocks of 1 / 4 MiB
        data = data * (4 if bid == 7 else 1)
    f = host(L.compress_frame(dev(data), L.make_sd(bid, sck, bck)))
    cap = len(data) + (4 << 20)
    (rs, os_), (rp, op_), (rf, of_) = _decode_all(f, cap)
    assert rs == rp == rf == 0 and os_ == op_ == of_ == data
    rng = random.Random(bid * 7 + sck * 3 + bck)
    bodies = [7 + rng.randrange(len(f) - 7) for _ in range(12)]
    cases = [f[:k] for k in bodies]                                   # truncations
    for k in bodies:                                                  # flipped bytes (size words, payload)
        bad = bytearray(f); bad[k] ^= 1 << rng.randrange(8); cases.append(bytes(bad))
    bad = bytearray(f); bad[7:11] = (0).to_bytes(4, "little"); cases.append(bytes(bad))          # early EOS
    bad = bytearray(f); bad[7:11] = ((1 << 24) | 5).to_bytes(4, "little"); cases.append(bytes(bad))  # > blockMax
    skip = (0x184D2A50).to_bytes(4, "little") + (3).to_bytes(4, "little") + b"abc"
    cases += [f + skip + f, f + f[:-3], f + b"xy"]
    for b in cases:
        (rs, os_), (rp, op_), (rf, of_) = _decode_all(b, 2 * cap)
        assert rs == rp == rf and os_ == op_ == of_, (len(b), rs, rp, rf)


def test_compress_frame_async_in_hip_graph(golden_inputs):
    """lz4mtHipCompressFrameAsync captured into a graph (torch.cuda.graph) and
    replayed gives the same frame as the direct call; outside a capture the
    block checksums run on a side stream, inside one they stay on the stream."""
    data = golden_inputs["syn300k"] * 4
    src = dev(data)
    sd = L.make_sd(4, False, True)
    want = host(L.compress_frame(src, sd))
    cap = L.frame_bound(src.numel(), sd)
    frame = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    fsz = torch.zeros(2, dtype=torch.int64, device="cuda")
    ws = L.compress_workspace(src.numel(), sd)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())

    def call():
        r = L.lib.lz4mtHipCompressFrameAsync(
            ctypes.c_void_p(src.data_ptr()), src.numel(), ctypes.c_void_p(frame.data_ptr()), cap,
            ctypes.c_void_p(fsz.data_ptr()), ctypes.byref(sd), ctypes.c_void_p(ws.data_ptr()), ws.numel(),
            ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert r == 0

    with torch.cuda.stream(s):   # warm-up outside the capture (side stream path)
        call()
    torch.cuda.synchronize()
    assert host(frame[:int(fsz[0].item())]) == want
    frame.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        call()
    g.replay()
    torch.cuda.synchronize()
    assert host(frame[:int(fsz[0].item())]) == want


def test_frame_engine_stream_size_field(golden_inputs):
    """FLG.3 through the device frame engine and the DEVICE host mode: same
    header as the reference writes (size + HC), same body, size reported back."""
    data = golden_inputs["syn300k"]
    plain = host(L.compress_frame(dev(data), L.make_sd(5, False, True)))
    sd = L.make_sd(5, False, True)
    sd.flg.streamSize = 1
    sd.streamSize = len(data)
    want = with_stream_size(plain, len(data))
    assert host(L.compress_frame(dev(data), sd)) == want
    r, frame = L.compress(data, sd, mode=L.MODE_DEVICE)
    assert r == 0 and frame == want
    out, r = L.decompress_frame(dev(want))
    assert r == 0 and host(out) == data
    r, out2, sd2 = L.decompress(want, len(data) + 64, mode=L.MODE_DEVICE)
    assert r == 0 and out2 == data and sd2.flg.streamSize == 1 and sd2.streamSize == len(data)


def test_block_decompress_fuzz_vs_oracle(golden_inputs):
    """Randomly damaged blocks (flipped bytes, truncations, appended or
    removed ranges) under several output caps: the GPU operator returns the
    same value as LZ4_decompress_safe 1.9.3 (the oracle; negative error
    positions included) and the same bytes when it succeeds."""
    rnd = random.Random(2024)
    syn = golden_inputs["syn300k"]
    srcs = [syn[:65536], syn[100_000:300_000], golden_inputs["text20k"],
            oracle.gen_random(5000, 3) + golden_inputs["zeros300k"][:50_000]]
    blocks = [oracle.compress_block(s, len(s) + len(s) // 255 + 16) for s in srcs]
    for it in range(2000):
        i = rnd.randrange(len(blocks))
        blk = bytearray(blocks[i])
        n = len(srcs[i])
        kind = rnd.randrange(5)
        if kind == 0:
            for _ in range(rnd.randrange(1, 5)):
                blk[rnd.randrange(len(blk))] = rnd.randrange(256)
        elif kind == 1:
            del blk[rnd.randrange(1, len(blk)):]
        elif kind == 2:
            blk += bytes(rnd.randrange(256) for _ in range(rnd.randrange(1, 40)))
        elif kind == 3:
            a = rnd.randrange(len(blk) - 1)
            del blk[a:a + rnd.randrange(1, 64)]
        else:
            a = rnd.randrange(len(blk) - 2)
            blk[a:a + 2] = rnd.randrange(65536).to_bytes(2, "little")
        cap = rnd.choice([n, n - 1, n + 100, max(1, n // 2), 4 << 20])
        got = L.decompress_block(bytes(blk), cap)
        want = oracle.decompress_block(bytes(blk), cap)
        assert got == want, (it, i, kind, cap, got[0], want[0])


@pytest.mark.parametrize("bid,sck,bck", [(4, True, True), (5, False, True), (7, True, False)])
def test_frame_decompress_fuzz_vs_oracle(golden_inputs, bid, sck, bck):
    """Randomly damaged frames through lz4mtHipDecompressFrame: the same
    Lz4MtResult as the oracle's restatement of lz4mt's decompress()
    (src/lz4mt.cpp:593-734, 938-1011), and the same bytes when it succeeds."""
    data = golden_inputs["syn300k"] + golden_inputs["random100k"] + golden_inputs["zeros300k"][:70_000]
    f = oracle.compress_frame(data, oracle.params(bid, sck, bck))
    rnd = random.Random(bid * 100 + sck * 10 + bck)
    cap = len(data) + (4 << 20)
    for it in range(150):
        b = bytearray(f)
        kind = rnd.randrange(4)
        if kind == 0:
            for _ in range(rnd.randrange(1, 4)):
                b[rnd.randrange(len(b))] ^= 1 << rnd.randrange(8)
        elif kind == 1:
            del b[rnd.randrange(4, len(b)):]
        elif kind == 2:
            a = rnd.randrange(7, len(b) - 4)
            b[a:a + 4] = rnd.randrange(1 << 32).to_bytes(4, "little")
        else:
            b += bytes(rnd.randrange(256) for _ in range(rnd.randrange(1, 12)))
        out = torch.empty(cap, dtype=torch.uint8, device="cuda")
        o, r = L.decompress_frame(dev(bytes(b)), out=out, check=False)
        rw, ow = oracle.decompress_frame(bytes(b), cap)
        assert r == rw, (it, kind, L.result_to_string(r), L.result_to_string(rw))
        if r == 0:
            assert host(o) == ow, (it, kind)


@pytest.mark.parametrize("mode", ["DEVICE", "PARALLEL", "PARALLEL_OPS"])
def test_callback_decompress_fuzz_vs_oracle(golden_inputs, mode):
    """The same damaged frames through lz4mtDecompress (callback API) in DEVICE
    and PARALLEL modes: the oracle's result code, and its bytes on success.
    What was written before an error is compared for DEVICE only: every block
    before the failing one, plus the failing block itself on a checksum
    mismatch (written before the check, src/lz4mt.cpp:665-681).  The
    reference's PARALLEL mode races there (tasks started after the quit skip
    their write), so only its result code is pinned."""
    m = {"DEVICE": L.MODE_DEVICE, "PARALLEL": L.MODE_PARALLEL, "PARALLEL_OPS": L.MODE_PARALLEL}[mode]
    # PARALLEL with null codecs runs the device engine; with the GPU block
    # operator set explicitly it runs block by block
    ops = (lambda src, dst, n, cap: L.lib.lz4mtHipDecompressBlock(src, dst, n, cap)) if mode == "PARALLEL_OPS" else None
    data = golden_inputs["syn300k"] + golden_inputs["random100k"]
    f = oracle.compress_frame(data, oracle.params(4, True, True))
    rnd = random.Random(77 if mode == "DEVICE" else 78)
    cap = len(data) + (1 << 20)
    for it in range(60):
        b = bytearray(f)
        kind = rnd.randrange(3)
        if kind == 0:
            b[rnd.randrange(len(b))] ^= 1 << rnd.randrange(8)
        elif kind == 1:
            del b[rnd.randrange(4, len(b)):]
        else:
            a = rnd.randrange(7, len(b) - 4)
            b[a:a + 4] = rnd.randrange(1 << 32).to_bytes(4, "little")
        r, out, _ = L.decompress(bytes(b), cap, mode=m, decompress_cb=ops)
        rw, ow = oracle.decompress_frame(bytes(b), cap)
        assert r == rw, (it, kind, L.result_to_string(r), L.result_to_string(rw))
        if r == 0 or mode != "PARALLEL_OPS":
            assert out == ow, (it, kind, L.result_to_string(r), len(out), len(ow))


# ---------------------------------------------------------------------------
# block checksums (k_xxh32_frame_blocks: 16 blocks per wave, a lane quad per
# block): ragged stored lengths (0-40 B and full 64 KiB), every byte
# alignment of the payload inside the frame, block counts that are not a
# multiple of 16; a flipped checksum word gives the oracle's result code
# ---------------------------------------------------------------------------
def _raw_block_frame(payloads, bad=None):
    import struct
    head = oracle.compress_frame(b"", oracle.params(4, False, True))[:-4]   # header only (no stream checksum)
    out = bytearray(head)
    for i, p in enumerate(payloads):
        ck = xxhash.xxh32(p).intdigest() ^ (1 if i == bad else 0)
        out += struct.pack("<I", len(p) | 0x80000000) + p + struct.pack("<I", ck)
    out += b"\0\0\0\0"
    return bytes(out)


@pytest.mark.parametrize("count", [1, 15, 17, 33, 50])
def test_block_checksums_ragged(count):
    rnd = random.Random(count)
    payloads = []
    for i in range(count):
        n = 65536 if i % 7 == 3 else rnd.randrange(1, 41)
        payloads.append(bytes(rnd.randrange(256) for _ in range(n)) if n < 100 else os.urandom(n))
    data = b"".join(payloads)
    for bad in (None, count // 2):
        fr = _raw_block_frame(payloads, bad)
        want_r, want = oracle.decompress_frame(fr, len(data) + 64)
        out, r = L.decompress_frame(dev(fr), check=False)
        assert r == want_r, (count, bad, r, want_r)
        assert (bad is not None) or host(out) == data == want
        r2, out2, _ = L.decompress(fr, len(data) + 64, mode=L.MODE_DEVICE)
        assert r2 == want_r and (bad is not None or out2 == data), (count, bad, r2)
