"""The streamed callback compress.

lz4mtCompress in MODE_DEVICE (and a relinked PARALLEL caller with null codec
callbacks) over independent 1 / 4 MiB blocks runs ONE persistent encoder grid
(k_encode_stream) that encodes each block as soon as read() has returned
it, while a writer thread writes the records in block order as they appear
(reference compress(), src/lz4mt.cpp:372-457: one read() per block, a read
of 0 ends the stream, write() per record piece).  Frames must be byte for
byte the batch engine's (LZ4MT_AMD_STREAM=0) and the App. F known answers;
the staging / output rings are forced tiny so they wrap thousands of times;
short reads are short blocks; a failing write() ends the call with an error
and the grid drains (the next call works)."""
import ctypes
import random
import struct

import pytest
import torch
import xxhash

import oracle

pytestmark = pytest.mark.gpu

L = None

APP_F = {  # SURVEY.md App. F, 256 MiB seed 42: (sck, bck, bid) -> (frame bytes, XXH32(frame))
    (1, 0, 7): (133159140, 0x157099A8), (0, 0, 7): (133159136, 0x8AC5DBC8), (1, 1, 7): (133159396, 0xC532D9D2),
    (0, 1, 7): (133159392, 0x1686045A), (1, 0, 6): (133770948, 0x7D1BC1BA), (0, 1, 6): (133771968, 0x535404A3),
    # round 6: 64 and 256 KiB blocks stream too (k_encode_stream's byU16 / v5 tables)
    (1, 0, 4): (131940148, 0xFC3A55A1), (0, 1, 5): (136145906, 0xE62BB3AC),
}


@pytest.fixture(scope="module", autouse=True)
def lib():
    global L
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    import lz4mt_amd
    L = lz4mt_amd
    return L


@pytest.fixture(scope="module")
def data256():
    d = oracle.gen_synthetic(256 << 20, 42)
    assert xxhash.xxh32(d).intdigest() == 0xE6F24EBA
    return d


@pytest.mark.parametrize("row", sorted(APP_F))
def test_streamed_known_answers(data256, row):
    sck, bck, bid = row
    r, frame = L.compress(data256, L.make_sd(bid, bool(sck), bool(bck)), mode=L.MODE_DEVICE)
    assert r == 0, L.result_to_string(r)
    assert (len(frame), xxhash.xxh32(frame).intdigest()) == APP_F[row], row
    r, out, _ = L.decompress(frame, len(data256) + 64, mode=L.MODE_DEVICE)
    assert r == 0 and xxhash.xxh32(out).intdigest() == 0xE6F24EBA


@pytest.mark.parametrize("rin,rout", [(8, 8), (9, 64), (256, 11)])
def test_streamed_tight_rings(data256, monkeypatch, rin, rout):
    """Staging and output rings of a few slots: the reader waits for pulls,
    the waves wait for the writer -- same bytes; the PARALLEL mode with null
    codecs takes the same engine."""
    monkeypatch.setenv("LZ4MT_AMD_STREAM_IN", str(rin))
    monkeypatch.setenv("LZ4MT_AMD_STREAM_OUT", str(rout))
    for row, m in (((0, 1, 6), L.MODE_DEVICE), ((1, 0, 7), L.MODE_PARALLEL), ((1, 0, 4), L.MODE_DEVICE)):
        sck, bck, bid = row
        r, frame = L.compress(data256, L.make_sd(bid, bool(sck), bool(bck)), mode=m)
        assert r == 0 and (len(frame), xxhash.xxh32(frame).intdigest()) == APP_F[row], (rin, rout, row)


def test_streamed_equals_batched(monkeypatch):
    """Mixed input (App. F text, incompressible stretches, zero runs; raw and
    compressed blocks) at 1 and 4 MiB blocks: the streamed frame is the batch
    engine's, byte for byte, and the oracle's."""
    rnd = random.Random(3)
    syn = oracle.gen_synthetic(40 << 20, 7)
    data = bytearray(syn)
    for s in range(0, len(data), 5 << 20):
        data[s:s + 1_500_000] = oracle.gen_random(1_500_000, s)
        z, k = s + 3_000_000, rnd.randrange(1, 900_000)
        data[z:z + k] = bytes(k)
    data = bytes(data[:(40 << 20) - 12345])
    for bid, sck, bck in ((6, True, True), (7, False, True), (6, False, False), (4, False, True), (5, True, True)):
        sd = L.make_sd(bid, sck, bck)
        r1, f1 = L.compress(data, sd, mode=L.MODE_DEVICE)
        monkeypatch.setenv("LZ4MT_AMD_STREAM", "0")
        r2, f2 = L.compress(data, sd, mode=L.MODE_DEVICE)
        monkeypatch.delenv("LZ4MT_AMD_STREAM")
        assert r1 == r2 == 0 and f1 == f2, (bid, sck, bck)
        assert f1 == oracle.compress_frame(data, oracle.params(bid, sck, bck)), (bid, sck, bck)


def _callbacks(data, sd, chunk_seed=None, fail_after=None):
    """lz4mtCompress in MODE_DEVICE with Python callbacks: random short reads
    (chunk_seed), or a write() that fails from its fail_after-th call on."""
    from lz4mt_amd import _abi
    rnd = random.Random(chunk_seed)
    src = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    st = {"pos": 0, "w": 0}
    reads, out = [], []

    def rd(ctx, dst, n):
        k = min(n, len(data) - st["pos"])
        if chunk_seed is not None and k > 1:
            k = rnd.choice([k, k, max(1, k // 3), rnd.randrange(1, k + 1)])
        ctypes.memmove(dst, ctypes.addressof(src) + st["pos"], k)
        st["pos"] += k
        reads.append(k)
        return k

    def wr(ctx, p, n):
        st["w"] += 1
        if fail_after is not None and st["w"] > fail_after:
            return -1
        out.append(ctypes.string_at(p, n))
        return n

    keep = [_abi.READ_FN(rd), _abi.WRITE_FN(wr)]
    ctx = L.init_context()
    ctx.mode = L.MODE_DEVICE
    ctx.read = ctypes.cast(keep[0], ctypes.c_void_p)
    ctx.write = ctypes.cast(keep[1], ctypes.c_void_p)
    r = L.lib.lz4mtCompress(ctypes.byref(ctx), ctypes.byref(sd))
    return r, b"".join(out), reads


def test_streamed_short_reads_are_short_blocks():
    data = oracle.gen_synthetic(30 << 20, 5)
    for bid, sck, bck, seed in ((6, True, True, 1), (7, False, True, 2)):
        r, frame, reads = _callbacks(data, L.make_sd(bid, sck, bck), chunk_seed=seed)
        assert r == 0, L.result_to_string(r)
        pieces, pos = [], 0
        for k in reads:
            if k:
                pieces.append(data[pos:pos + k])
                pos += k
        bm = 1 << (8 + 2 * bid)
        assert pos == len(data) and any(len(p) < bm for p in pieces[:-1])
        head = oracle.compress_frame(b"", oracle.params(bid, sck, bck))[:7]
        want = bytearray(head)
        for p in pieces:
            c = oracle.compress_block(p, len(p))
            stored = c if c else p
            want += struct.pack("<I", len(c) if c else len(p) | 0x80000000) + stored
            if bck:
                want += struct.pack("<I", xxhash.xxh32(stored).intdigest())
        want += b"\0\0\0\0"
        if sck:
            want += struct.pack("<I", xxhash.xxh32(data).intdigest())
        assert frame == bytes(want), (bid, sck, bck)


def test_streamed_empty_and_tiny_inputs():
    for data in (b"", b"x", oracle.gen_synthetic(1 << 20, 3), oracle.gen_synthetic((1 << 20) + 5, 3)):
        sd = L.make_sd(6, True, True)
        r, frame, _ = _callbacks(data, sd)
        assert r == 0 and frame == oracle.compress_frame(data, oracle.params(6, True, True)), len(data)


def test_streamed_write_failure_drains():
    """write() fails part-way: the call returns an error (no hang, the grid
    drains), the records before it were written, and the next call is fine."""
    data = oracle.gen_synthetic(64 << 20, 9)
    sd = L.make_sd(6, False, True)
    r, frame, _ = _callbacks(data, sd, fail_after=40)
    assert r != 0
    want = oracle.compress_frame(data, oracle.params(6, False, True))
    assert want.startswith(frame) and len(frame) > 7
    r, frame, _ = _callbacks(data, sd)
    assert r == 0 and frame == want


# ---------------------------------------------------------------------------
# The streamed decompress (k_decode_stream): lz4mtDecompress in MODE_DEVICE
# (and PARALLEL with a null decompress callback) over independent 1 / 4 MiB
# blocks decodes each record as soon as it is read; same bytes and result
# codes as the batch engine (LZ4MT_AMD_STREAM=0) and the oracle.
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("row", sorted(APP_F))
def test_streamed_decompress_known_answers(data256, row):
    sck, bck, bid = row
    frame = oracle.compress_frame(data256[:64 << 20], oracle.params(bid, bool(sck), bool(bck)))
    for m in (L.MODE_DEVICE, L.MODE_PARALLEL):
        r, out, sd = L.decompress(frame, (64 << 20) + 64, mode=m)
        assert r == 0, (row, m, L.result_to_string(r))
        assert out == data256[:64 << 20], (row, m)


@pytest.mark.parametrize("rin,rout", [(8, 8), (9, 64), (256, 11)])
def test_streamed_decompress_tight_rings(data256, monkeypatch, rin, rout):
    monkeypatch.setenv("LZ4MT_AMD_STREAM_IN", str(rin))
    monkeypatch.setenv("LZ4MT_AMD_STREAM_OUT", str(rout))
    for row in ((0, 1, 6), (1, 1, 7)):
        sck, bck, bid = row
        frame = oracle.compress_frame(data256[:48 << 20], oracle.params(bid, bool(sck), bool(bck)))
        r, out, _ = L.decompress(frame, (48 << 20) + 64, mode=L.MODE_DEVICE)
        assert r == 0 and out == data256[:48 << 20], (rin, rout, row)


def _damaged_frames(seed):
    """Frames with raw and compressed blocks (1 MiB), then damaged: a flipped
    byte in a compressed block, in a raw block, in a block checksum, in the
    stream checksum; a size word past blockMax; truncations inside a size
    word, a block and a checksum; a missing EOS."""
    rnd = random.Random(seed)
    data = bytearray(oracle.gen_synthetic(9 << 20, seed))
    data[3 << 20:(3 << 20) + 900_000] = oracle.gen_random(900_000, seed)   # an incompressible stretch: raw blocks
    data = bytes(data)
    out = []
    for sck, bck in ((True, True), (False, True), (True, False)):
        f = oracle.compress_frame(data, oracle.params(6, sck, bck))
        out.append(("intact", sck, bck, f))
        recs, pos = [], 7
        while True:   # walk the records
            w = struct.unpack_from("<I", f, pos)[0]
            if w == 0:
                break
            n = w & 0x7FFFFFFF
            recs.append((pos, w, n))
            pos += 4 + n + (4 if bck else 0)
        comp = [r_ for r_ in recs if not r_[1] & 0x80000000]
        raw = [r_ for r_ in recs if r_[1] & 0x80000000]
        p0, _, n0 = comp[rnd.randrange(len(comp))]
        g = bytearray(f)
        g[p0 + 4 + rnd.randrange(n0)] ^= 0x5A
        out.append(("flip-compressed", sck, bck, bytes(g)))
        if raw:
            p1, _, n1 = raw[0]
            g = bytearray(f)
            g[p1 + 4 + n1 // 2] ^= 1
            out.append(("flip-raw", sck, bck, bytes(g)))
        if bck:
            g = bytearray(f)
            g[p0 + 4 + n0] ^= 1
            out.append(("flip-checksum", sck, bck, bytes(g)))
        if sck:
            g = bytearray(f)
            g[-1] ^= 1
            out.append(("flip-stream-checksum", sck, bck, bytes(g)))
        g = bytearray(f)
        struct.pack_into("<I", g, recs[2][0], (1 << 20) + 1)
        out.append(("size-past-blockmax", sck, bck, bytes(g)))
        out.append(("cut-size-word", sck, bck, f[:recs[3][0] + 2]))
        out.append(("cut-block", sck, bck, f[:recs[3][0] + 4 + recs[3][2] // 2]))
        if bck:
            out.append(("cut-checksum", sck, bck, f[:recs[3][0] + 4 + recs[3][2] + 2]))
        out.append(("no-eos", sck, bck, f[:pos]))
    return data, out


def test_streamed_decompress_damaged_frames_match_batch_engine(monkeypatch):
    """Every damaged frame gives the batch engine's result code and the same
    bytes written before the error, in MODE_DEVICE."""
    data, frames = _damaged_frames(11)
    for label, sck, bck, f in frames:
        r1, o1, _ = L.decompress(f, len(data) + 64, mode=L.MODE_DEVICE)
        monkeypatch.setenv("LZ4MT_AMD_STREAM", "0")
        r2, o2, _ = L.decompress(f, len(data) + 64, mode=L.MODE_DEVICE)
        monkeypatch.delenv("LZ4MT_AMD_STREAM")
        assert (r1, o1) == (r2, o2), (label, sck, bck, L.result_to_string(r1), L.result_to_string(r2))
        if label == "intact":
            assert r1 == 0 and o1 == data


def test_streamed_decompress_concatenated_and_after_error():
    """Two frames back to back decode as one stream; a failing call leaves
    the grid drained (the next call works)."""
    a = oracle.gen_synthetic(6 << 20, 1)
    b = oracle.gen_synthetic(5 << 20, 2)
    fa = oracle.compress_frame(a, oracle.params(6, True, True))
    fb = oracle.compress_frame(b, oracle.params(7, False, True))
    r, out, _ = L.decompress(fa + fb, len(a) + len(b) + 64, mode=L.MODE_DEVICE)
    assert r == 0 and out == a + b
    bad = bytearray(fa)
    bad[7 + 4 + 100] ^= 0xFF
    r, _, _ = L.decompress(bytes(bad), len(a) + 64, mode=L.MODE_DEVICE)
    assert r != 0
    r, out, _ = L.decompress(fb, len(b) + 64, mode=L.MODE_DEVICE)
    assert r == 0 and out == b


def test_streamed_decompress_random_frames_vs_batch_engine(monkeypatch):
    """40 random frames (1 / 4 MiB blocks, every flag combination, sizes up to
    20 MiB with raw stretches and zero runs), a third of them damaged at a
    random byte or cut at a random length: the streamed decompress gives the
    batch engine's result code and bytes, and the oracle's bytes when intact."""
    rnd = random.Random(2024)
    for case in range(40):
        bid = rnd.choice((6, 7))
        sck, bck, ssz = rnd.random() < 0.5, rnd.random() < 0.5, rnd.random() < 0.3
        n = rnd.randrange(1, 20 << 20)
        data = bytearray(oracle.gen_synthetic(n, case))
        if n > 4 << 20 and rnd.random() < 0.5:
            z = rnd.randrange(n - (2 << 20))
            data[z:z + (1 << 20)] = oracle.gen_random(1 << 20, case)
        if n > 1 << 20 and rnd.random() < 0.3:
            z = rnd.randrange(n - (1 << 20))
            data[z:z + (1 << 20)] = bytes(1 << 20)
        data = bytes(data)
        f = oracle.compress_frame(data, oracle.params(bid, sck, bck, n if ssz else None))
        kind = rnd.random()
        if kind < 0.17:
            g = bytearray(f)
            g[rnd.randrange(7, len(g))] ^= 1 << rnd.randrange(8)
            f = bytes(g)
        elif kind < 0.33:
            f = f[:rnd.randrange(7, len(f))]
        r1, o1, _ = L.decompress(f, n + 64, mode=L.MODE_DEVICE)
        monkeypatch.setenv("LZ4MT_AMD_STREAM", "0")
        r2, o2, _ = L.decompress(f, n + 64, mode=L.MODE_DEVICE)
        monkeypatch.delenv("LZ4MT_AMD_STREAM")
        assert (r1, o1) == (r2, o2), (case, bid, sck, bck, ssz, n, kind, L.result_to_string(r1), L.result_to_string(r2))
        if kind >= 0.33:
            assert r1 == 0 and o1 == data, (case, L.result_to_string(r1))


def _slow_io(fn, data, sd, mode, slow_read=None, slow_write=None, delay=2.5):
    """lz4mtCompress / lz4mtDecompress with Python callbacks, one of which
    blocks for `delay` seconds at its slow_read-th / slow_write-th call (a
    stalled pipe upstream or downstream)."""
    import time
    from lz4mt_amd import _abi
    src = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    st = {"pos": 0, "r": 0, "w": 0}
    out = []

    def rd(ctx, dst, n):
        st["r"] += 1
        if st["r"] == slow_read:
            time.sleep(delay)
        k = min(n, len(data) - st["pos"])
        ctypes.memmove(dst, ctypes.addressof(src) + st["pos"], k)
        st["pos"] += k
        return k

    def wr(ctx, p, n):
        st["w"] += 1
        if st["w"] == slow_write:
            time.sleep(delay)
        out.append(ctypes.string_at(p, n))
        return n

    keep = [_abi.READ_FN(rd), _abi.WRITE_FN(wr)]
    ctx = L.init_context()
    ctx.mode = mode
    ctx.read = ctypes.cast(keep[0], ctypes.c_void_p)
    ctx.write = ctypes.cast(keep[1], ctypes.c_void_p)
    r = fn(ctypes.byref(ctx), ctypes.byref(sd))
    return r, b"".join(out)


def test_streamed_slow_callbacks_are_not_a_timeout(monkeypatch):
    """With the grids' wait limit at 1 s (LZ4MT_AMD_STREAM_TIMEOUT_S), a read()
    or write() that blocks 2.5 s (the whole grid waiting on it) still ends in
    the right frame / bytes: time inside a callback is progress (the
    keepalive word), only a host that stops without being in one times out."""
    monkeypatch.setenv("LZ4MT_AMD_STREAM_TIMEOUT_S", "1")
    monkeypatch.setenv("LZ4MT_AMD_STREAM_IN", "8")
    monkeypatch.setenv("LZ4MT_AMD_STREAM_OUT", "8")
    data = oracle.gen_synthetic(24 << 20, 4)
    want = oracle.compress_frame(data, oracle.params(6, True, True))
    for slow in ({"slow_read": 3}, {"slow_write": 12}):
        r, frame = _slow_io(L.lib.lz4mtCompress, data, L.make_sd(6, True, True), L.MODE_DEVICE, **slow)
        assert r == 0 and frame == want, (slow, L.result_to_string(r))
    for slow in ({"slow_read": 9}, {"slow_write": 4}):
        r, out = _slow_io(L.lib.lz4mtDecompress, want, L.init_stream_descriptor(), L.MODE_DEVICE, **slow)
        assert r == 0 and out == data, (slow, L.result_to_string(r))


def test_streamed_concurrent_calls_from_threads():
    """Three host threads compress and decompress at once in MODE_DEVICE
    (each thread's call launches its own persistent grid; grids that share a
    hardware queue or the CUs run one after the other): every frame and
    every decode is right, nothing waits on another call."""
    import threading
    inputs = [oracle.gen_synthetic((9 << 20) + 777 * k, 20 + k) for k in range(3)]
    sds = [(6, True, True), (7, False, True), (6, False, False)]
    res = [None] * 3

    def work(k):
        try:
            bid, sck, bck = sds[k]
            r, frame = L.compress(inputs[k], L.make_sd(bid, sck, bck), mode=L.MODE_DEVICE)
            r2, out, _ = L.decompress(frame, len(inputs[k]) + 64, mode=L.MODE_DEVICE)
            res[k] = (r, frame, r2, out)
        except Exception as e:   # reported below
            res[k] = e

    ths = [threading.Thread(target=work, args=(k,)) for k in range(3)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(240)
    for k in range(3):
        assert not isinstance(res[k], Exception) and res[k] is not None, (k, res[k])
        r, frame, r2, out = res[k]
        bid, sck, bck = sds[k]
        assert r == 0 and frame == oracle.compress_frame(inputs[k], oracle.params(bid, sck, bck)), k
        assert r2 == 0 and out == inputs[k], k


def _rss_bytes():
    with open("/proc/self/statm") as f:
        import os
        return int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE")


def test_streamed_rings_freed_at_thread_exit():
    """A DEVICE-mode call keeps its streamed rings (pinned host memory, ~0.8
    GiB at 1 MiB blocks) per thread for the next call; a thread that exits
    frees them: four short-lived threads in turn leave the resident set where
    the first one left it."""
    import threading
    data = oracle.gen_synthetic(3 << 20, 8)
    sd = L.make_sd(6, False, True)

    def one():
        r, _ = L.compress(data, sd, mode=L.MODE_DEVICE)
        assert r == 0

    rss = []
    for _ in range(4):
        t = threading.Thread(target=one)
        t.start()
        t.join(120)
        rss.append(_rss_bytes())
    assert rss[-1] - rss[0] < (512 << 20), [x >> 20 for x in rss]


def test_read_callback_claiming_more_than_asked():
    """A read() that returns more than the n bytes it was asked for (a broken
    callback) is taken as n bytes: no engine reads or copies past its
    buffers; streamed DEVICE, batch DEVICE and PARALLEL frames all hold the
    bytes actually delivered, n per read."""
    from lz4mt_amd import _abi
    data = oracle.gen_synthetic(5 << 20, 12)
    for mode, stream in ((L.MODE_DEVICE, "1"), (L.MODE_DEVICE, "0"), (L.MODE_PARALLEL, "0")):
        src = ctypes.create_string_buffer(data, len(data))
        st = {"pos": 0}
        out = []

        def rd(ctx, dst, n):
            k = min(n, len(data) - st["pos"])
            ctypes.memmove(dst, ctypes.addressof(src) + st["pos"], k)
            st["pos"] += k
            return k + 4096 if k else 0   # claims 4 KiB more than it wrote

        def wr(ctx, p, n):
            out.append(ctypes.string_at(p, n))
            return n

        import os
        old = os.environ.get("LZ4MT_AMD_STREAM")
        os.environ["LZ4MT_AMD_STREAM"] = stream
        try:
            keep = [_abi.READ_FN(rd), _abi.WRITE_FN(wr)]
            ctx = L.init_context()
            ctx.mode = mode
            ctx.read = ctypes.cast(keep[0], ctypes.c_void_p)
            ctx.write = ctypes.cast(keep[1], ctypes.c_void_p)
            sd = L.make_sd(6, True, True)
            r = L.lib.lz4mtCompress(ctypes.byref(ctx), ctypes.byref(sd))
        finally:
            if old is None:
                del os.environ["LZ4MT_AMD_STREAM"]
            else:
                os.environ["LZ4MT_AMD_STREAM"] = old
        assert r == 0, (mode, stream, L.result_to_string(r))
        assert b"".join(out) == oracle.compress_frame(data, oracle.params(6, True, True)), (mode, stream)


def _dec_fail_write(frame, fail_at):
    """lz4mtDecompress in MODE_DEVICE with a write() that fails at its
    fail_at-th call; returns (result, bytes written before it)."""
    from lz4mt_amd import _abi
    src = ctypes.create_string_buffer(frame, len(frame))
    st = {"pos": 0, "w": 0}
    out = []

    def rd(ctx, dst, n):
        k = min(n, len(frame) - st["pos"])
        ctypes.memmove(dst, ctypes.addressof(src) + st["pos"], k)
        st["pos"] += k
        return k

    def wr(ctx, p, n):
        st["w"] += 1
        if st["w"] == fail_at:
            return n - 1
        out.append(ctypes.string_at(p, n))
        return n

    keep = [_abi.READ_FN(rd), _abi.WRITE_FN(wr)]
    ctx = L.init_context()
    ctx.mode = L.MODE_DEVICE
    ctx.read = ctypes.cast(keep[0], ctypes.c_void_p)
    ctx.write = ctypes.cast(keep[1], ctypes.c_void_p)
    sd = L.init_stream_descriptor()
    r = L.lib.lz4mtDecompress(ctypes.byref(ctx), ctypes.byref(sd))
    return r, b"".join(out)


def test_streamed_decompress_write_failure(monkeypatch):
    """A write() that fails on a decoded block and on a raw (stored) block:
    the streamed decompress ends with the batch engine's result code
    (CANNOT_WRITE_DECODED_BLOCK / CANNOT_WRITE_DATA_BLOCK, the reference's
    codes) and the same bytes before it; the grid drains and the next call
    decodes the whole frame."""
    data = bytearray(oracle.gen_synthetic(12 << 20, 31))
    data[5 << 20:6 << 20] = oracle.gen_random(1 << 20, 31)   # block 5 is stored raw
    data = bytes(data)
    frame = oracle.compress_frame(data, oracle.params(6, True, True))
    want = {3: L.Result.CANNOT_WRITE_DECODED_BLOCK, 6: L.Result.CANNOT_WRITE_DATA_BLOCK}
    for k, code in want.items():
        r1, o1 = _dec_fail_write(frame, k)
        monkeypatch.setenv("LZ4MT_AMD_STREAM", "0")
        r2, o2 = _dec_fail_write(frame, k)
        monkeypatch.delenv("LZ4MT_AMD_STREAM")
        assert (r1, o1) == (r2, o2), (k, L.result_to_string(r1), L.result_to_string(r2))
        assert r1 == code, (k, L.result_to_string(r1))
        assert o1 == data[:(k - 1) << 20], k
    r, out = _dec_fail_write(frame, None)
    assert r == 0 and out == data


@pytest.mark.parametrize("bid,sck,bck", [(6, True, True), (6, False, True), (7, True, False)])
def test_streamed_decompress_damaged_vs_oracle(bid, sck, bck):
    """Randomly damaged 1 / 4 MiB-block frames through the streamed
    decompress (lz4mtDecompress, MODE_DEVICE): the oracle's result code
    (its restatement of src/lz4mt.cpp:593-734, 938-1011) and the oracle's
    bytes -- on success, and the bytes written before an error."""
    rnd = random.Random(bid * 100 + sck * 10 + bck)
    n = (9 << 20) + 4321 if bid == 7 else (3 << 20) + 777
    data = bytearray(oracle.gen_synthetic(n, bid))
    data[n // 3:n // 3 + 300_000] = oracle.gen_random(300_000, bid)
    data = bytes(data)
    f = oracle.compress_frame(data, oracle.params(bid, sck, bck))
    cap = n + (4 << 20)
    for it in range(40 if bid == 6 else 16):
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
        r, out, _ = L.decompress(bytes(b), cap, mode=L.MODE_DEVICE)
        rw, ow = oracle.decompress_frame(bytes(b), cap)
        assert r == rw, (it, kind, L.result_to_string(r), L.result_to_string(rw))
        assert out == ow, (it, kind, L.result_to_string(r), len(out), len(ow))


def _hook_io(fn, data, sd, hooks, whooks=None):
    """lz4mtCompress / lz4mtDecompress (MODE_DEVICE) with Python callbacks;
    hooks[k] runs inside the k-th read() call (1-based) before it returns,
    whooks[k] inside the k-th write() call."""
    from lz4mt_amd import _abi
    src = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    st = {"pos": 0, "r": 0, "w": 0}
    out = []
    whooks = whooks or {}

    def rd(ctx, dst, n):
        st["r"] += 1
        if st["r"] in hooks:
            hooks[st["r"]]()
        k = min(n, len(data) - st["pos"])
        ctypes.memmove(dst, ctypes.addressof(src) + st["pos"], k)
        st["pos"] += k
        return k

    def wr(ctx, p, n):
        st["w"] += 1
        if st["w"] in whooks:
            whooks[st["w"]]()
        out.append(ctypes.string_at(p, n))
        return n

    keep = [_abi.READ_FN(rd), _abi.WRITE_FN(wr)]
    ctx = L.init_context()
    ctx.mode = L.MODE_DEVICE
    ctx.read = ctypes.cast(keep[0], ctypes.c_void_p)
    ctx.write = ctypes.cast(keep[1], ctypes.c_void_p)
    r = fn(ctypes.byref(ctx), ctypes.byref(sd))
    return r, b"".join(out)


def _lds_heavy_gpu_work():
    """GPU work that needs LDS (a GEMM and a radix sort), waited for."""
    a = torch.randn(2048, 2048, device="cuda")
    x = torch.sort(torch.rand(1 << 22, device="cuda"))[0]
    return float((a @ a).sum().item()) + float(x[-1].item())


def test_streamed_reader_stall_parks_the_grid(monkeypatch, capfd):
    """A read() that stalls past LZ4MT_AMD_STREAM_PARK_MS parks the streamed
    grid: its waiting waves leave the device, so GPU work that needs LDS --
    here launched and waited for INSIDE the stalled read() -- runs (the grid
    holds every CU's LDS while it waits, so without parking this callback
    could never return); the reader then relaunches the grid at the next
    block and the frames and bytes are exact.  Compress and decompress,
    stalls early and late, a stall in the final read() (no relaunch), tight
    rings."""
    import time
    monkeypatch.setenv("LZ4MT_AMD_STREAM_PARK_MS", "50")
    monkeypatch.setenv("LZ4MT_AMD_PIPE_TRACE", "1")
    # every CU's LDS held by the grid (the default, 4 waves per CU, leaves
    # half of it free, and the callback's GPU work would not need the park)
    monkeypatch.setenv("LZ4MT_AMD_STREAM_WAVES_PER_CU", "8")
    waits = []

    def timed_work():
        t = time.time()
        _lds_heavy_gpu_work()
        waits.append(time.time() - t)

    _lds_heavy_gpu_work()   # warm-up: libraries loaded, kernels compiled
    data = oracle.gen_synthetic(24 << 20, 41)
    frame = oracle.compress_frame(data, oracle.params(6, True, True))
    for rings in ((256, 512), (8, 8)):
        monkeypatch.setenv("LZ4MT_AMD_STREAM_IN", str(rings[0]))
        monkeypatch.setenv("LZ4MT_AMD_STREAM_OUT", str(rings[1]))
        for hooks in ({3: timed_work}, {2: timed_work, 17: timed_work},
                      {25: lambda: time.sleep(0.2)}):   # read 25 returns 0: a stall at the end
            t0 = time.time()
            r, got = _hook_io(L.lib.lz4mtCompress, data, L.make_sd(6, True, True), hooks)
            assert r == 0 and got == frame, (rings, sorted(hooks), L.result_to_string(r))
            assert time.time() - t0 < 60
        # decompress: three read() calls per record (size word, data, checksum)
        for hooks in ({4: timed_work}, {2: timed_work, 30: timed_work}):
            r, got = _hook_io(L.lib.lz4mtDecompress, frame, L.init_stream_descriptor(), hooks)
            assert r == 0 and got == data, (rings, sorted(hooks), L.result_to_string(r))
    err = capfd.readouterr().err
    relaunches = err.count("relaunched at block")
    with capfd.disabled():
        print(f"hook waits (s): {[round(w, 3) for w in waits]}; relaunches: {relaunches}")
    # every hook that ran while a grid was up had to wait for the park (>= 50 ms)
    assert relaunches >= 8 and sum(w >= 0.045 for w in waits) >= 8, (waits, relaunches)


def test_streamed_writer_stall_parks_the_grid(monkeypatch, capfd):
    """VERDICT r05 item 4 / ADVICE r05: a write() that stalls past
    LZ4MT_AMD_STREAM_PARK_MS parks the grid too.  Waves whose block is done
    but whose output slot is taken leave it in their HBM buffers (a pend
    descriptor per wave), waiting waves leave, the reader publishes nothing
    meanwhile; GPU work that needs LDS -- launched and waited for INSIDE the
    stalled write() -- runs; when the write() returns the grid is relaunched
    and every parked block goes out first.  With 8 waves per CU (every CU's
    LDS held) this callback could not return without the park.  Compress and
    decompress, tight rings (the output ring full while the writer stalls),
    stalls early and late, a read() and a write() stalled at once."""
    import time
    monkeypatch.setenv("LZ4MT_AMD_STREAM_PARK_MS", "50")
    monkeypatch.setenv("LZ4MT_AMD_STREAM_WAVES_PER_CU", "8")
    monkeypatch.setenv("LZ4MT_AMD_PIPE_TRACE", "1")
    waits = []

    def timed_work():
        t = time.time()
        _lds_heavy_gpu_work()
        waits.append(time.time() - t)

    def slow_then_work():
        time.sleep(0.1)
        timed_work()

    _lds_heavy_gpu_work()
    data = oracle.gen_synthetic(24 << 20, 43)
    frame = oracle.compress_frame(data, oracle.params(6, True, True))
    for rings in ((256, 512), (8, 8)):
        monkeypatch.setenv("LZ4MT_AMD_STREAM_IN", str(rings[0]))
        monkeypatch.setenv("LZ4MT_AMD_STREAM_OUT", str(rings[1]))
        # compress: three write() calls per record (size word, payload, checksum) after the header's
        # the reader is kept busy (10 ms per read(), below the park threshold),
        # so the grid's idle waves sit in their input waits -- holding the LDS
        # -- while the writer stalls, as in a real pipe
        for rh, wh in (({}, {2: timed_work}), ({}, {5: timed_work, 40: timed_work}),
                       ({6: slow_then_work}, {8: timed_work}), ({}, {62: timed_work})):
            rh = {**{k: (lambda: time.sleep(0.01)) for k in range(1, 26)}, **rh}
            t0 = time.time()
            r, got = _hook_io(L.lib.lz4mtCompress, data, L.make_sd(6, True, True), rh, wh)
            assert r == 0 and got == frame, (rings, sorted(wh), L.result_to_string(r))
            assert time.time() - t0 < 60
        # decompress: one write() per decoded block
        for rh, wh in (({}, {1: timed_work}), ({}, {3: timed_work, 14: timed_work}),
                       ({10: slow_then_work}, {4: timed_work}), ({}, {18: timed_work})):
            rh = {**{k: (lambda: time.sleep(0.01)) for k in range(2, 75, 3)}, **rh}   # the data reads
            r, got = _hook_io(L.lib.lz4mtDecompress, frame, L.init_stream_descriptor(), rh, wh)
            assert r == 0 and got == data, (rings, sorted(wh), L.result_to_string(r))
    err = capfd.readouterr().err
    relaunches = err.count("relaunched at block")
    with capfd.disabled():
        print(f"write-hook waits (s): {[round(w, 3) for w in waits]}; relaunches: {relaunches}")
    assert "a write() stalled" in err, err[-2000:]
    # the hooks that ran while idle waves held the LDS waited for the park
    assert relaunches >= 8 and sum(w >= 0.045 for w in waits) >= 8, (waits, relaunches)


def test_streamed_compress_piped_into_streamed_decompress(monkeypatch):
    """two streamed calls of one process joined by a pipe on one
    GPU (compress | decompress), every CU's LDS held by whichever grid runs
    (8 waves per CU), tiny rings and a pipe far smaller than the data: each
    grid parks while its write() / read() waits on the other, so the pair
    completes instead of hanging; bytes exact."""
    import os
    import threading
    from lz4mt_amd import _abi
    monkeypatch.setenv("LZ4MT_AMD_STREAM_PARK_MS", "50")
    monkeypatch.setenv("LZ4MT_AMD_STREAM_WAVES_PER_CU", "8")
    monkeypatch.setenv("LZ4MT_AMD_STREAM_IN", "8")
    monkeypatch.setenv("LZ4MT_AMD_STREAM_OUT", "8")
    data = oracle.gen_synthetic(40 << 20, 44)
    src = ctypes.create_string_buffer(bytes(data), len(data))
    rfd, wfd = os.pipe()
    pos = {"c": 0}
    out = []
    res = {}

    def c_read(ctx, dst, n):
        k = min(n, len(data) - pos["c"])
        ctypes.memmove(dst, ctypes.addressof(src) + pos["c"], k)
        pos["c"] += k
        return k

    def c_write(ctx, p, n):
        b = ctypes.string_at(p, n)
        while b:
            b = b[os.write(wfd, b):]
        return n

    def d_read(ctx, dst, n):
        got = 0
        while got < n:
            b = os.read(rfd, n - got)
            if not b:
                break
            ctypes.memmove(dst + got, b, len(b))
            got += len(b)
        return got

    def d_write(ctx, p, n):
        out.append(ctypes.string_at(p, n))
        return n

    keep = [_abi.READ_FN(c_read), _abi.WRITE_FN(c_write), _abi.READ_FN(d_read), _abi.WRITE_FN(d_write)]

    def run(kind):
        ctx = L.init_context()
        ctx.mode = L.MODE_DEVICE
        if kind == "c":
            ctx.read, ctx.write = ctypes.cast(keep[0], ctypes.c_void_p), ctypes.cast(keep[1], ctypes.c_void_p)
            res["c"] = L.lib.lz4mtCompress(ctypes.byref(ctx), ctypes.byref(L.make_sd(6, True, True)))
            os.close(wfd)
        else:
            ctx.read, ctx.write = ctypes.cast(keep[2], ctypes.c_void_p), ctypes.cast(keep[3], ctypes.c_void_p)
            res["d"] = L.lib.lz4mtDecompress(ctypes.byref(ctx), ctypes.byref(L.init_stream_descriptor()))
    th = [threading.Thread(target=run, args=(k,), daemon=True) for k in "cd"]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    alive = any(t.is_alive() for t in th)
    os.close(rfd)
    assert not alive, "compress | decompress through a pipe did not finish"
    assert res == {"c": 0, "d": 0}, res
    assert b"".join(out) == data
