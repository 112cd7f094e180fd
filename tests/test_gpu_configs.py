"""GPU parity at the BASELINE.json sizes and through the callback engine.

* Known answers for configs[1] (8 GiB, 4 MiB blocks, -Sx -BX), the default
  flags at 8 GiB, configs[2] (32 GiB: frame and record offsets past 2^32) and
  a 10 GiB 1 MiB-block frame (the parallel walk past 2^32), computed by the
  pinned oracle (tests/golden/make_known_answers.py): frame size, XXH32 of
  the frame (8 GiB cases) and the chunked checksum of checksums of the frame
  and of the decoded content.
* The multi-batch DEVICE / default-PARALLEL callback engine (many batches,
  slot reuse, in-order writer) against the SURVEY.md App. F known answers.
* Reference callback semantics: short reads (a short read is a short block,
  src/lz4mt.cpp:435-450), write() per record piece (src/lz4mt.cpp:418-428),
  frames cut inside a size or checksum word, FILE* bindings
  (src/lz4mt_io_cstdio.cpp) on the GPU engines.
"""
import ctypes
import os
import random
import struct
import threading

import pytest
import torch
import xxhash

import oracle
from conftest import checksum_of_checksums

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


def host(t):
    return bytes(t.cpu().numpy().tobytes())


# ---------------------------------------------------------------------------
# large configs against the oracle's known answers
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("case", ["configs1_8gib_b7_SxBX", "8gib_b7_default", "configs2_32gib_b7_SxBX",
                                  "10gib_b6_SxBX", "8gib_b5_SxBX", "8gib_b4_SxBX"])
def test_known_answers_large(known_answers, case):
    ka = known_answers["cases"][case]
    chunk = known_answers["chunk"]
    n = ka["bytes"]
    src = L.gen_synthetic(n, seed=known_answers["seed"])
    assert checksum_of_checksums(src, chunk) == ka["content_chunks"]
    sd = L.make_sd(ka["block_id"], ka["stream_checksum"], ka["block_checksum"])
    frame = L.compress_frame(src, sd)
    assert frame.numel() == ka["frame_size"], (case, frame.numel())
    assert checksum_of_checksums(frame, chunk) == ka["frame_chunks"], case
    if n <= 8 << 30:   # the one-wave serial XXH32 over the whole frame
        assert L.xxh32(frame) == ka["frame_xxh32"], case
    del src
    torch.cuda.empty_cache()
    out, r = L.decompress_frame(frame)
    assert r == 0 and out.numel() == n, (case, r, out.numel())
    assert checksum_of_checksums(out, chunk) == ka["content_chunks"], case
    # the record table walks past 2^32 where the frame does
    if ka["frame_size"] > 1 << 32:
        hl, recs, _ = L.frame_records(frame)
        assert recs[-1] == ka["frame_size"] - 4 and recs[-2] > 1 << 32
    del out, frame
    torch.cuda.empty_cache()


# ---------------------------------------------------------------------------
# the callback engine over many batches
# ---------------------------------------------------------------------------
APP_F = {  # SURVEY.md App. F, 256 MiB seed 42: (sck, bck, bid) -> (frame bytes, XXH32(frame))
    (1, 0, 7): (133159140, 0x157099A8), (0, 1, 7): (133159392, 0x1686045A), (1, 0, 4): (131940148, 0xFC3A55A1),
    (0, 1, 5): (136145906, 0xE62BB3AC), (1, 0, 6): (133770948, 0x7D1BC1BA),
}


@pytest.fixture(scope="module")
def data256():
    d = oracle.gen_synthetic(256 << 20, 42)
    assert xxhash.xxh32(d).intdigest() == 0xE6F24EBA
    return d


@pytest.fixture
def small_batches(monkeypatch):
    # 16 MiB first batch, batches capped at 32 MiB, two slots: ~9 batches per
    # 256 MiB frame, every slot reused several times
    monkeypatch.setenv("LZ4MT_AMD_BATCH0_MIB", "16")
    monkeypatch.setenv("LZ4MT_AMD_BATCH_MIB", "32")
    monkeypatch.setenv("LZ4MT_AMD_SLOTS", "2")
    # the batch engine (every block size streams by default since round 6)
    monkeypatch.setenv("LZ4MT_AMD_STREAM", "0")


@pytest.mark.parametrize("mode", ["DEVICE", "PARALLEL"])
@pytest.mark.parametrize("row", sorted(APP_F))
def test_multibatch_engine_known_answers(data256, small_batches, mode, row):
    m = L.MODE_DEVICE if mode == "DEVICE" else L.MODE_PARALLEL   # PARALLEL + null codecs = the batch engine
    sck, bck, bid = row
    r, frame = L.compress(data256, L.make_sd(bid, bool(sck), bool(bck)), mode=m)
    assert r == 0, L.result_to_string(r)
    assert (len(frame), xxhash.xxh32(frame).intdigest()) == APP_F[row], (mode, row)
    r, out, sd = L.decompress(frame, len(data256) + 64, mode=m)
    assert r == 0 and len(out) == len(data256) and xxhash.xxh32(out).intdigest() == 0xE6F24EBA, (mode, row)
    assert (sd.bd.blockMaximumSize, sd.flg.streamChecksum, sd.flg.blockChecksum) == (bid, sck, bck)


# ---------------------------------------------------------------------------
# raw callbacks: short reads, write pieces
# ---------------------------------------------------------------------------
def _run_callbacks(fn, data, sd, mode, chunk=None, compress_cb=None, decompress_cb=None, seed=1):
    """Runs lz4mtCompress/lz4mtDecompress with Python read/write callbacks.
    ``chunk``: the reader returns random short counts (1..n) until EOF.
    Returns (result, output bytes, [sizes returned by read], [sizes of write calls])."""
    from lz4mt_amd import _abi
    rnd = random.Random(seed)
    src = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    st = {"pos": 0, "eof": 0}
    reads, writes, out = [], [], []

    def rd(ctx, dst, n):
        k = min(n, len(data) - st["pos"])
        if chunk and k > 1:
            k = rnd.choice([k, max(1, k // 3), rnd.randrange(1, k + 1)])
        if k < n:
            st["eof"] = int(st["pos"] + k >= len(data))
        ctypes.memmove(dst, ctypes.addressof(src) + st["pos"], k)
        st["pos"] += k
        reads.append(k)
        return k

    def eof(ctx):
        return st["eof"]

    def wr(ctx, p, n):
        out.append(ctypes.string_at(p, n))
        writes.append(n)
        return n

    keep = [_abi.READ_FN(rd), _abi.READ_EOF_FN(eof), _abi.WRITE_FN(wr)]
    ctx = L.init_context()
    ctx.mode = mode
    ctx.read = ctypes.cast(keep[0], ctypes.c_void_p)
    ctx.readEof = ctypes.cast(keep[1], ctypes.c_void_p)
    ctx.write = ctypes.cast(keep[2], ctypes.c_void_p)
    if compress_cb is not None:
        keep.append(_abi.COMPRESS_FN(compress_cb))
        ctx.compress = ctypes.cast(keep[-1], ctypes.c_void_p)
    if decompress_cb is not None:
        keep.append(_abi.DECOMPRESS_FN(decompress_cb))
        ctx.decompress = ctypes.cast(keep[-1], ctypes.c_void_p)
    r = fn(ctypes.byref(ctx), ctypes.byref(sd))
    return r, b"".join(out), reads, writes


def _frame_of_pieces(pieces, bid, sck, bck):
    """The frame lz4mt writes when read() returns these pieces (each one a
    block, src/lz4mt.cpp:435-450): oracle block codec, cap = piece size."""
    head = oracle.compress_frame(b"", oracle.params(bid, sck, bck))[:7]
    out = bytearray(head)
    for p in pieces:
        c = oracle.compress_block(p, len(p))
        stored = c if c else p
        out += struct.pack("<I", len(c) if c else len(p) | 0x80000000) + stored
        if bck:
            out += struct.pack("<I", xxhash.xxh32(stored).intdigest())
    out += b"\0\0\0\0"
    if sck:
        out += struct.pack("<I", xxhash.xxh32(b"".join(pieces)).intdigest())
    return bytes(out)


@pytest.mark.parametrize("mode", ["DEVICE", "PARALLEL"])
def test_short_reads_are_short_blocks(golden_inputs, mode):
    m = L.MODE_DEVICE if mode == "DEVICE" else L.MODE_PARALLEL
    data = (golden_inputs["syn300k"] + golden_inputs["zeros300k"] + golden_inputs["random100k"]) * 2
    for bid, sck, bck, seed in ((4, True, True, 1), (5, False, True, 2), (6, True, False, 3)):
        r, frame, reads, _ = _run_callbacks(L.lib.lz4mtCompress, data, L.make_sd(bid, sck, bck), m, chunk=True,
                                            seed=seed)
        assert r == 0, L.result_to_string(r)
        pieces, pos = [], 0
        for k in reads:
            if k:
                pieces.append(data[pos:pos + k])
                pos += k
        bm = 1 << (8 + 2 * bid)
        assert pos == len(data) and any(len(p) < bm for p in pieces[:-1])   # short blocks before the last
        assert frame == _frame_of_pieces(pieces, bid, sck, bck), (mode, bid)
        r, out, _ = L.decompress(frame, len(data) + (1 << 20), mode=m)
        assert r == 0 and out == data


def test_write_pieces_match_the_reference(golden_inputs):
    """The DEVICE engine calls write() per record in the reference's pieces
    (size word, payload, checksum word), like the per-block host engine."""
    data = golden_inputs["syn300k"] + golden_inputs["random100k"]
    sd = L.make_sd(4, True, True)
    ops = lambda s, d, n, c, lv: L.lib.lz4mtHipCompressBlock(s, d, n, c, lv)   # noqa: E731
    r1, f1, _, w1 = _run_callbacks(L.lib.lz4mtCompress, data, sd, L.MODE_DEVICE)
    r2, f2, _, w2 = _run_callbacks(L.lib.lz4mtCompress, data, sd, L.MODE_PARALLEL, compress_cb=ops)
    assert r1 == r2 == 0 and f1 == f2 == oracle.compress_frame(data, oracle.params(4, True, True))
    assert w1 == w2
    nb = (len(data) + 65535) // 65536
    assert len(w1) == 1 + 3 * nb + 2 and w1[0] == 7 and w1[1] == 4 and w1[-2:] == [4, 4]
    assert max(w1) <= 65536


def _words(frame, bck):
    """(size-word offsets, checksum-word offsets) of a single frame's records."""
    from lz4mt_amd import dist as D
    hdr, recs, end = D.walk_records(frame, block_checksum=bck)
    return [a for a, _ in recs] + [end - 4], [b - 4 for _, b in recs] if bck else []


def test_truncated_inside_words_device_mode(golden_inputs):
    """Frames cut inside a mid-batch size word or block checksum word: the
    oracle's result code (CANNOT_READ_BLOCK_SIZE / _CHECKSUM), and every block
    before the cut written (DEVICE mode reads those words without setting
    ERROR, so the batched blocks are still written)."""
    data = golden_inputs["syn300k"] + golden_inputs["zeros300k"]
    f = oracle.compress_frame(data, oracle.params(4, False, True))
    sizes, cks = _words(f, True)
    cases = [f[:o + k] for o in sizes[3:-1:2] for k in (1, 2, 3)] + [f[:o + 2] for o in cks[2::3]]
    cases += [f[:sizes[-1] + 2]]   # inside the EOS word
    for b in cases:
        r, out, _ = L.decompress(b, len(data) + (1 << 20), mode=L.MODE_DEVICE)
        rw, ow = oracle.decompress_frame(b, len(data) + (1 << 20))
        assert r == rw and r in (L.Result.CANNOT_READ_BLOCK_SIZE, L.Result.CANNOT_READ_BLOCK_CHECKSUM), \
            (len(b), L.result_to_string(r), L.result_to_string(rw))
        assert out == ow, (len(b), len(out), len(ow))


# ---------------------------------------------------------------------------
# FILE* bindings (lz4mtIoBindCstdio, reference src/lz4mt_io_cstdio.cpp) on the GPU
# ---------------------------------------------------------------------------
def _file_run(fn, src, dst, mode, sd=None):
    ctx = L.init_context()
    ctx.mode = mode
    L.lib.lz4mtIoBindCstdio(ctypes.byref(ctx))
    assert L.lib.lz4mtIoOpenIstream(ctypes.byref(ctx), str(src).encode())
    assert L.lib.lz4mtIoOpenOstream(ctypes.byref(ctx), str(dst).encode(), 0)
    sd = sd if sd is not None else L.init_stream_descriptor()
    r = fn(ctypes.byref(ctx), ctypes.byref(sd))
    L.lib.lz4mtIoCloseIstream(ctypes.byref(ctx))
    L.lib.lz4mtIoCloseOstream(ctypes.byref(ctx))
    return r, sd


@pytest.mark.parametrize("mode", ["DEVICE", "PARALLEL"])
def test_cstdio_files_on_gpu(tmp_path, mode):
    m = L.MODE_DEVICE if mode == "DEVICE" else L.MODE_PARALLEL
    data = oracle.gen_synthetic(37 << 20, 9) + oracle.gen_random(3 << 20, 4) + bytes(1 << 20) + b"tail"
    src, mid, back = tmp_path / "in.bin", tmp_path / "in.lz4", tmp_path / "back.bin"
    src.write_bytes(data)
    for bid, sck, bck in ((7, True, False), (5, False, True), (6, True, True)):
        r, _ = _file_run(L.lib.lz4mtCompress, src, mid, m, L.make_sd(bid, sck, bck))
        assert r == 0, L.result_to_string(r)
        assert mid.read_bytes() == oracle.compress_frame(data, oracle.params(bid, sck, bck)), (mode, bid)
        r, sd = _file_run(L.lib.lz4mtDecompress, mid, back, m)
        assert r == 0 and back.read_bytes() == data, (mode, bid, L.result_to_string(r))
        assert sd.bd.blockMaximumSize == bid


# ---------------------------------------------------------------------------
# resources: the block operators' scratch pool, the stream bound
# ---------------------------------------------------------------------------
def test_block_operator_threads_do_not_leak():
    """The reference runs each block on a fresh std::async thread
    (src/lz4mt.cpp:448): many short-lived threads calling the operators must
    not accumulate device memory."""
    blk = oracle.gen_synthetic(1 << 20, 5)
    want = oracle.compress_block(blk, len(blk))

    def one(res):
        dst = ctypes.create_string_buffer(len(blk) + 64)
        n = L.lib.lz4mtHipCompressBlock(blk, dst, len(blk), len(blk), 0)
        res.append(dst.raw[:n] == want)
        out = ctypes.create_string_buffer(4 << 20)
        res.append(L.lib.lz4mtHipDecompressBlock(dst, out, n, 4 << 20) == len(blk))

    def wave(k):
        res = []
        th = [threading.Thread(target=one, args=(res,)) for _ in range(k)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert all(res) and len(res) == 2 * k

    wave(8)
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    for _ in range(25):
        wave(8)
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info()[0]
    assert free0 - free1 < (64 << 20), (free0, free1)
    L.lib.lz4mtHipReleaseCaches()


def test_decompress_frame_sizes_concatenated_frames(golden_inputs):
    a, b = golden_inputs["syn300k"], golden_inputs["zeros300k"]
    fa = oracle.compress_frame(a, oracle.params(4, True, True))
    fb = oracle.compress_frame(b, oracle.params(7, False, False))
    skip = (0x184D2A5F).to_bytes(4, "little") + (3).to_bytes(4, "little") + b"xyz"
    t = torch.frombuffer(bytearray(fa + skip + fb + fa), dtype=torch.uint8).cuda()
    assert L.stream_bound(t) >= 2 * len(a) + len(b)
    out, r = L.decompress_frame(t)   # sized by lz4mtHipStreamBound
    assert r == 0 and host(out) == a + b + a
