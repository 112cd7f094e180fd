"""Multi-process (gloo, world_size 2 and 3) tests of the block-sharded frame
path (lz4mt_amd/dist.py) -- the same gather / scatter /
verify orchestration bench.py runs over RCCL at N > 1.  CPU only: each rank
compresses its block range with the oracle (the checker), the record runs
are gathered over torch.distributed, and the stitched frame must equal the
oracle's frame of the whole stream byte for byte; the root then scatters
that frame back and every rank decodes its own block range."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from lz4mt_amd import dist as D


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, block_id, bck, q, async_op=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = oracle.gen_synthetic(n, 42)
        bm = D.block_bytes(block_id)
        off, ln, _, _ = D.shard_blocks(n, bm, world, rank)
        p = oracle.params(block_id, stream_checksum=False, block_checksum=bck)
        local = oracle.compress_frame(data[off:off + ln], p)
        t = torch.frombuffer(bytearray(local + b"\xAA" * 13), dtype=torch.uint8)   # slack past the frame end
        if async_op:   # enqueue, do other work reading the frame, then wait (bench.py at N > 1)
            full, works = D.gather_frame(t, len(local), async_op=True)
            assert oracle.decompress_frame(bytes(t.numpy().tobytes())[:len(local)], ln + bm)[1] == data[off:off + ln]
            for w in works:
                w.wait()
        else:
            full = D.gather_frame(t, len(local))
        if rank == 0:
            q.put(bytes(full.numpy().tobytes()))
    finally:
        dist.destroy_process_group()


def _run(world, n, block_id, bck, async_op=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, block_id, bck, q, async_op)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


@pytest.mark.parametrize("n,block_id,bck,async_op", [(17 * 65536 + 12345, 4, True, False),
                                                     (3 * 262144, 5, False, False),
                                                     (17 * 65536 + 12345, 4, True, True)])
def test_gather_stitches_whole_stream_frame(n, block_id, bck, async_op):
    got = _run(2, n, block_id, bck, async_op)
    want = oracle.compress_frame(oracle.gen_synthetic(n, 42), oracle.params(block_id, False, bck))
    assert got == want


def test_gather_more_ranks_than_blocks():
    # 3 ranks, 2 blocks: one rank owns an empty shard (a header + EOS frame)
    n = 65536 + 100
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 3, port, n, 4, True, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == oracle.compress_frame(oracle.gen_synthetic(n, 42), oracle.params(4, False, True))


def test_shard_plan_covers_stream():
    for n, bm, world in [(0, 65536, 2), (1, 65536, 3), (10 * 65536, 65536, 4), (10 * 65536 + 7, 65536, 8),
                         (8 << 30, 4 << 20, 8)]:
        pos = 0
        for r in range(world):
            off, ln, first, count = D.shard_blocks(n, bm, world, r)
            assert off == pos and (off % bm == 0 or off == n)
            assert ln <= count * bm
            pos += ln
        assert pos == n


@pytest.mark.parametrize("world", [1, 2, 3, 5])
def test_split_frame_decodes_to_slices(world):
    n = 9 * 65536 + 333
    data = oracle.gen_synthetic(n, 7)
    frame = oracle.compress_frame(data, oracle.params(4, False, True))
    parts = D.split_frame(frame, world)
    out = b""
    for r, part in enumerate(parts):
        rc, dec = oracle.decompress_frame(part, n + 65536)
        assert rc == 0
        off, ln, _, _ = D.shard_blocks(n, 65536, world, r)
        assert dec == data[off:off + ln]
        out += dec
    assert out == data
    # and the pieces stitch back into the original frame
    hdr, _, _ = D.walk_records(frame)
    assert frame[:hdr] + b"".join(p[hdr:-4] for p in parts) + D.EOS == frame


def test_stream_checksum_frames_refuse_to_shard():
    frame = oracle.compress_frame(oracle.gen_synthetic(70000, 1), oracle.params(4, True, False))
    with pytest.raises(ValueError, match="serial"):
        D.split_frame(frame, 2)


def _digests(t, chunk=1 << 16):
    import xxhash
    b = t.numpy().tobytes()
    return torch.tensor([xxhash.xxh32(b[i:i + chunk]).intdigest() for i in range(0, len(b), chunk)],
                        dtype=torch.int64)


def _oracle_decode(cap):
    """A frame (CPU uint8 tensor) -> its content (the stitched frame's per-shard pieces in verify_stitched)."""
    def dec(f):
        out = oracle.decompress_frame(f.numpy().tobytes(), cap)[1]
        return torch.frombuffer(bytearray(out) or bytearray(1), dtype=torch.uint8)[:len(out)]
    return dec


def _roundtrip_worker(rank, world, port, n, block_id, q, corrupt_rank=None):
    """bench.py's N > 1 step on the CPU: local frame -> gather to root ->
    verify the stitched frame against every shard -> scatter it back ->
    decode the own piece."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = oracle.gen_synthetic(n, 42)
        bm = D.block_bytes(block_id)
        off, ln, _, _ = D.shard_blocks(n, bm, world, rank)
        shard = data[off:off + ln]
        p = oracle.params(block_id, stream_checksum=False, block_checksum=True)
        local = oracle.compress_frame(shard, p)
        full = D.gather_frame(torch.frombuffer(bytearray(local), dtype=torch.uint8), len(local))
        src = bytearray(shard)
        if rank == corrupt_rank and src:
            src[len(src) // 2] ^= 1
        ok = D.verify_stitched(full, torch.frombuffer(src, dtype=torch.uint8) if src else torch.zeros(0, dtype=torch.uint8),
                               decode=_oracle_decode(n + bm),
                               digests=_digests)
        piece = D.scatter_frame(full if rank == 0 else None, full.numel() if rank == 0 else 0)
        rc, dec = oracle.decompress_frame(piece.numpy().tobytes(), ln + bm)
        q.put((rank, ok, rc == 0 and dec == shard, piece.numel()))
    finally:
        dist.destroy_process_group()


def _run_roundtrip(world, n, block_id, corrupt_rank=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_roundtrip_worker, args=(r, world, port, n, block_id, q, corrupt_rank))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world,n,block_id", [(2, 17 * 65536 + 12345, 4), (3, 7 * 262144 + 5, 5), (3, 65536 + 9, 4),
                                             (4, 9 * 65536 + 3, 4)])
def test_gather_verify_scatter_roundtrip(world, n, block_id):
    res = _run_roundtrip(world, n, block_id)
    assert all(ok for _, ok, _, _ in res), res           # stitched frame matches every shard
    assert all(dec for _, _, dec, _ in res), res         # each scattered piece decodes to its shard


def test_verify_stitched_catches_a_bad_shard():
    res = _run_roundtrip(2, 9 * 65536, 4, corrupt_rank=1)
    assert not any(ok for _, ok, _, _ in res), res


def test_scatter_pieces_are_the_shard_frames():
    """The pieces the scatter makes are byte for byte the frames each rank
    would write for its own shard (same header, its records, EOS)."""
    n, bid, world = 11 * 65536 + 77, 4, 3
    data = oracle.gen_synthetic(n, 42)
    p = oracle.params(bid, False, True)
    frame = oracle.compress_frame(data, p)
    hdr, starts = D.host_records(torch.frombuffer(bytearray(frame), dtype=torch.uint8))
    for r in range(world):
        first, count = D.rank_blocks(len(starts) - 1, world, r)
        off, ln, _, _ = D.shard_blocks(n, 65536, world, r)
        piece = frame[:hdr] + frame[starts[first]:starts[first + count]] + D.EOS
        assert piece == oracle.compress_frame(data[off:off + ln], p)


def test_stream_size_frames_refuse_to_shard():
    frame = oracle.compress_frame(oracle.gen_synthetic(70000, 1), oracle.params(4, False, True, stream_size=70000))
    with pytest.raises(ValueError, match="FLG.3"):
        D.split_frame(frame, 2)


def _error_worker(rank, world, port, kind, q):
    """A frame the source rank cannot cut (-BD, or damaged so the walk runs
    off its end) must make EVERY rank raise, not leave the others waiting in
    the broadcast (scatter) or the all_gather (gather)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = oracle.gen_synthetic(5 * 65536, 3)
        good = oracle.compress_frame(data, oracle.params(4, False, True))
        if kind == "bd":   # FLG.5 clear: a block-dependent frame does not shard
            bad = bytearray(good)
            bad[4] &= ~0x20
            bad = bytes(bad)
        else:   # a size word pointing past the frame end
            bad = bytearray(good)
            bad[7:11] = (0x7FFFFF00).to_bytes(4, "little")
            bad = bytes(bad)
        try:
            if kind == "gather":   # rank 1 holds a shard frame with a damaged magic word
                f = (b"\x05" + good[1:]) if rank == 1 else good
                D.gather_frame(torch.frombuffer(bytearray(f), dtype=torch.uint8), len(f))
            else:
                t = torch.frombuffer(bytearray(bad), dtype=torch.uint8)
                D.scatter_frame(t if rank == 0 else None, len(bad) if rank == 0 else 0)
            q.put((rank, "returned"))
        except (ValueError, RuntimeError) as e:
            q.put((rank, "raised: " + str(e)[:60]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["bd", "damaged", "gather"])
def test_bad_frame_raises_on_every_rank(kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_error_worker, args=(r, 2, port, kind, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1].startswith("raised") for r in res), res


# ---------------------------------------------------------------------------
# compress_gather_streamed: the round protocol on the CPU with a mock engine
# ---------------------------------------------------------------------------
class MockShardEngine:
    """CPU stand-in for dist.HipShardEngine (test infrastructure): the same
    pack wire format (lz4mt_shard.hip: 64-byte header, 16-byte descriptor
    per block, stored sizes, block checksums, payload at a 256-byte
    boundary), the encoder's output taken from the oracle (the checker) and
    published a little more every round, at a per-block pace, so blocks
    finish out of step; the encode of rank r ends after `2 + r` rounds.
    Blocks that end incompressible first publish bytes that are NOT their
    stored bytes (the device encoder publishes a prefix before it gives
    up), so the last round's switch to the source bytes is exercised."""

    def __init__(self, rank, bid, rounds_to_finish):
        self.bm = 1 << (8 + 2 * bid)
        self.rounds_to_finish = rounds_to_finish
        self.calls = 0

    def header(self, sd):
        import lz4mt_amd as L   # host-only code of the library: no device needed
        return L.frame_header(sd)

    def workspace(self, n, sd):
        nb = (n + self.bm - 1) // self.bm
        return {"n": n, "nb": nb, "slots": [bytearray(self.bm) for _ in range(nb)], "csize": [0] * nb,
                "bsum": [0] * nb, "sent": [0] * nb}

    def pack_buffer(self, n, sd, cap):
        nb = (n + self.bm - 1) // self.bm
        return torch.zeros(self._data_off(nb) + nb * min(cap, self.bm) + 64, dtype=torch.uint8)

    @staticmethod
    def _data_off(nb):
        return (64 + 24 * nb + 255) & ~255

    def encode(self, src, sd, ws):
        import xxhash
        data = bytes(src.numpy().tobytes())
        self.src, self.final, self.pace = data, [], []
        for b in range(ws["nb"]):
            blk = data[b * self.bm:(b + 1) * self.bm]
            c = oracle.compress_block(blk, len(blk))   # cap = n (src/lz4mt.cpp:391)
            cs = len(c) if c else 0
            ws["csize"][b] = cs
            ws["bsum"][b] = xxhash.xxh32(c if cs else blk).intdigest()
            self.final.append(c if cs else b"\xEE" * (len(blk) // 3))   # a raw block's abandoned prefix
            self.pace.append(1 + (b * 7919) % 5)

    def encode_finished(self):
        return self.calls >= self.rounds_to_finish

    def _published(self, b):
        f = self.final[b]
        return min(len(f), len(f) * self.calls * self.pace[b] // (4 * self.rounds_to_finish))

    def pack(self, src, sd, ws, buf, cap, final):
        import struct
        nb, raw_bit = ws["nb"], 0x80000000
        cap = min(cap, self.bm)
        b0 = bytearray(buf.numel())
        doff, off, rem, body = self._data_off(nb), 0, 0, 0
        for b in range(nb):
            n_b = min(self.bm, ws["n"] - b * self.bm)
            s = ws["sent"][b]
            raw = False
            if final:
                cs = ws["csize"][b]
                if cs > 0:
                    hi, srcb = cs, self.final[b]
                else:
                    if not s & raw_bit:
                        s = raw_bit
                    raw, hi, srcb = True, n_b, self.src[b * self.bm:b * self.bm + n_b]
                body += 4 + (cs if cs > 0 else n_b) + (4 if sd.flg.blockChecksum else 0)
                struct.pack_into("<i", b0, 64 + 16 * nb + 4 * b, cs)
                struct.pack_into("<I", b0, 64 + 20 * nb + 4 * b, ws["bsum"][b] if sd.flg.blockChecksum else 0)
            else:
                hi, srcb = self._published(b), self.final[b]
            lo = s & ~raw_bit
            avail = max(hi - lo, 0)
            ln = min(avail, cap)
            struct.pack_into("<IIQ", b0, 64 + 16 * b, lo | (raw_bit if raw else 0), ln, off)
            b0[doff + off:doff + off + ln] = srcb[lo:lo + ln]
            ws["sent"][b] = (raw_bit if raw else 0) | (lo + ln)
            off += ln
            rem += avail - ln
        flags = 1 if final and rem == 0 else 0
        struct.pack_into("<QQQQIIQ", b0, 0, 0x44485354344D5A4C, off, rem, doff + off, nb, flags, body if final else 0)
        buf.copy_(torch.frombuffer(b0, dtype=torch.uint8))
        self.calls += 1
        return D.parse_pack_header(bytes(b0[:64]))

    def unpack(self, buf, n, sd, mirror):
        import struct
        b0 = bytes(buf.numpy().tobytes())
        nb = mirror["nb"]
        flags = struct.unpack_from("<I", b0, 36)[0]
        doff = self._data_off(nb)
        for b in range(nb):
            lo, ln, off = struct.unpack_from("<IIQ", b0, 64 + 16 * b)
            lo &= 0x7FFFFFFF
            mirror["slots"][b][lo:lo + ln] = b0[doff + off:doff + off + ln]
            if flags & 1:
                mirror["csize"][b] = struct.unpack_from("<i", b0, 64 + 16 * nb + 4 * b)[0]
                mirror["bsum"][b] = struct.unpack_from("<I", b0, 64 + 20 * nb + 4 * b)[0]

    def _records(self, src, ws, sd):
        import struct
        out = bytearray()
        for b in range(ws["nb"]):
            n_b = min(self.bm, ws["n"] - b * self.bm)
            cs = ws["csize"][b]
            if src is not None:   # the rank's own shard: its encoder output / source
                pay = self.final[b] if cs > 0 else self.src[b * self.bm:b * self.bm + n_b]
            else:
                pay = bytes(ws["slots"][b][:cs if cs > 0 else n_b])
            out += struct.pack("<I", cs if cs > 0 else (n_b | 0x80000000)) + pay
            if sd.flg.blockChecksum:
                out += struct.pack("<I", ws["bsum"][b])
        return bytes(out)

    def body_bytes(self, n, sd, ws):
        return len(self._records(self.src, ws, sd))

    def assemble(self, src, n, sd, ws, body):
        rec = self._records(src if src is None else self.src, ws, sd)
        assert len(rec) == body.numel()
        body.copy_(torch.frombuffer(bytearray(rec), dtype=torch.uint8) if rec else body)


def _streamed_worker(rank, world, port, n, block_id, bck, kind, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import lz4mt_amd as L
        data = _stream_input(n, kind)
        bm = D.block_bytes(block_id)
        off, ln, _, _ = D.shard_blocks(n, bm, world, rank)
        sd = L.make_sd(block_id, stream_checksum=False, block_checksum=bck)
        eng = MockShardEngine(rank, block_id, 2 + rank)
        stats = {}
        full = D.compress_gather_streamed(torch.frombuffer(bytearray(data[off:off + ln]) or bytearray(1),
                                                           dtype=torch.uint8)[:ln], sd, engine=eng,
                                          per_block_cap=max(bm // 8, 4096), stats=stats, min_round_s=0.0)
        if rank == 0:
            q.put((bytes(full.numpy().tobytes()), stats["rounds"]))
    finally:
        dist.destroy_process_group()


def _stream_input(n, kind):
    if kind == "mixed":   # compressible text with incompressible stretches: some blocks stored raw
        a = bytearray(oracle.gen_synthetic(n, 42))
        r = oracle.gen_random(n, 9)
        for s in range(0, n, 3 * 65536 + 1000):
            a[s:s + 70000] = r[s:s + 70000]
        return bytes(a)
    return oracle.gen_synthetic(n, 42)


@pytest.mark.parametrize("world,n,block_id,bck,kind", [
    (2, 9 * 65536 + 4321, 4, True, "appf"),
    (3, 23 * 65536 + 77, 4, False, "mixed"),
    (3, 2 * 262144, 5, True, "mixed"),          # 2 blocks, 3 ranks: one shard is empty
    (2, 3 * (1 << 20) + 5, 6, True, "mixed"),
])
def test_streamed_gather_stitches_whole_stream_frame(world, n, block_id, bck, kind):
    """compress_gather_streamed over gloo: ranks finish their encodes in
    different rounds, blocks publish at different paces, payloads are capped
    per block per round (several final rounds), incompressible blocks switch
    to source bytes -- and the root's frame is byte for byte the oracle's
    frame of the whole stream."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_streamed_worker, args=(r, world, port, n, block_id, bck, kind, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got, rounds = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = oracle.compress_frame(_stream_input(n, kind), oracle.params(block_id, False, bck))
    assert rounds > world + 1
    assert got == want


def _layout_worker(rank, world, port, q):
    """A shard that is not a whole number of blocks, followed by another
    shard: the stitched frame would not be the whole stream's, so EVERY
    rank raises, none waits in a round."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import lz4mt_amd as L
        bm = D.block_bytes(4)
        ln = bm + 100 if rank == 0 else 2 * bm
        sd = L.make_sd(4, stream_checksum=False, block_checksum=True)
        eng = MockShardEngine(rank, 4, 2)
        try:
            D.compress_gather_streamed(torch.frombuffer(bytearray(oracle.gen_synthetic(ln, 3)), dtype=torch.uint8),
                                       sd, engine=eng, min_round_s=0.0)
            q.put((rank, "no error"))
        except ValueError as e:
            q.put((rank, str(e)))
    finally:
        dist.destroy_process_group()


def test_streamed_gather_rejects_ragged_inner_shard():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_layout_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all("not whole" in m for _, m in res), res


def test_ipc_layout_key_tracks_every_field():
    """IpcPushTransport keeps its buffers only for the same shard sizes,
    descriptor, per-block cap and root."""
    import lz4mt_amd as L
    sd6, sd7 = L.make_sd(6, False, True), L.make_sd(7, False, True)
    k = D.IpcPushTransport._layout_key
    base = k([8 << 20, 8 << 20], sd7, 1 << 17, 0)
    assert base == k([8 << 20, 8 << 20], L.make_sd(7, False, True), 1 << 17, 0)
    for other in (k([8 << 20, 12 << 20], sd7, 1 << 17, 0), k([8 << 20, 8 << 20], sd6, 1 << 17, 0),
                  k([8 << 20, 8 << 20], sd7, 1 << 16, 0), k([8 << 20, 8 << 20], sd7, 1 << 17, 1)):
        assert other != base
