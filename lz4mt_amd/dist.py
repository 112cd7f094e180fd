"""Block-sharded multi-GPU frames.

lz4mt frames with independent blocks (FLG bit 5, reference
src/lz4mt.cpp:914-918) are a header, a run of self-delimiting block records
(u32 size word | payload | [u32 block XXH32]) and an EOS word
(src/lz4mt.cpp:418-428, 923-925).  A record depends only on its own block,
so a stream cut at block boundaries can be compressed shard by shard on
different GPUs and the record runs concatenated: the result is byte-for-byte
the frame one process would write for the whole stream.  The one thing that
does not shard is the stream (content) checksum, a single serial XXH32 chain
(SURVEY.md §0.5), so sharded frames require FLG.2 = 0 (``-Sx``).

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm,
"gloo" for CPU tests).  Compress: each rank encodes its contiguous block
range locally, then the compressed record runs are gathered to the root (the
only exchange step of the path, ``gather_frame``).  Decompress of one frame
across ranks (``scatter_frame``): the root walks the size words on the
device (lz4mtHipFrameRecords, O(blocks)), cuts the record table at the
ranks' block ranges and sends each rank its run of whole records with
grouped point-to-point transfers; each rank decodes header + records + EOS
locally.  ``verify_stitched`` checks a stitched frame against every rank's
source (root decode, per-shard chunk digests).
"""
import ctypes
import struct

import torch
import torch.distributed as dist

MAGIC = 0x184D2204
SKIPPABLE_MIN, SKIPPABLE_MAX = 0x184D2A50, 0x184D2A5F
EOS = b"\x00\x00\x00\x00"


def block_bytes(block_max_id):
    """getBlockSize (reference src/lz4mt.cpp:34-37)."""
    if not 4 <= block_max_id <= 7:
        raise ValueError(f"block maximum size id {block_max_id} not in [4, 7]")
    return 1 << (8 + 2 * block_max_id)


def shard_blocks(n_total, bm, world, rank):
    """Contiguous block range of ``rank``: returns (byte offset, byte length, first block, block count).

    Blocks [0, nb) are split as evenly as possible; the last (short) block
    goes to the last rank that owns blocks.
    """
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    nb = (n_total + bm - 1) // bm
    per, rem = divmod(nb, world)
    first = rank * per + min(rank, rem)
    count = per + (1 if rank < rem else 0)
    off = min(first * bm, n_total)
    end = min((first + count) * bm, n_total)
    return off, end - off, first, count


def header_length(flg):
    """Frame header bytes after the magic word: FLG, BD, [u64 size], [u32 dict], HC (src/lz4mt.cpp:335-369)."""
    return 3 + (8 if flg & 0x08 else 0) + (4 if flg & 0x01 else 0)


def _frame_layout(head):
    """(header length incl. magic, FLG) from the first bytes of a frame."""
    if len(head) < 6 or struct.unpack_from("<I", head, 0)[0] != MAGIC:
        raise ValueError("not an lz4mt frame (magic)")
    flg = head[4]
    if not flg & 0x20:
        raise ValueError("block-dependent frames (-BD) do not shard")
    if flg & 0x04:
        raise ValueError("a stream checksum (FLG.2) is one serial chain and cannot be sharded; use -Sx")
    if flg & 0x08:
        # the content-size field (and the header checksum over it) describes
        # one shard, not the stitched stream, nor a piece of a split frame
        raise ValueError("a content-size field (FLG.3) does not survive sharding; leave streamSize unset")
    return 4 + header_length(flg), flg


def frame_records(frame, frame_len=None):
    """(header length, records length) of a single -Sx frame held in a uint8 tensor or bytes."""
    frame_len = len(frame) if frame_len is None else int(frame_len)
    head = bytes(frame[:20].cpu().numpy().tobytes()) if isinstance(frame, torch.Tensor) else bytes(frame[:20])
    hdr, _ = _frame_layout(head)
    rec = frame_len - hdr - 4
    if rec < 0:
        raise ValueError("frame shorter than header + EOS")
    return hdr, rec


def gather_frame(frame, frame_len, dst=0, group=None, async_op=False):
    """Gathers every rank's shard frame into ONE frame on ``dst``.

    ``frame`` is this rank's uint8 tensor (device tensor under RCCL, CPU under
    gloo) holding a complete -Sx frame of ``frame_len`` bytes.  Ranks must
    hold consecutive block ranges in rank order (``shard_blocks``) and equal
    frame headers.  Returns the stitched frame on ``dst`` (header of rank 0,
    record runs in rank order, EOS) and None elsewhere.

    Exchange: one all_gather of the record-run lengths (8 B per rank), then
    grouped point-to-point sends of each rank's record run straight into its
    final place in the root's frame (no padding, no staging copy).  This is
    the path's only collective; it is bound by the root's inbound xGMI links.

    With ``async_op`` the point-to-point transfers are only enqueued: the
    call returns ``(frame_or_None, works)`` and the caller waits on
    ``works`` (e.g. after launching the local decompress, which only reads
    ``frame``); the stitched frame is complete once they are done.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    err = None
    try:
        hdr, rec = frame_records(frame, frame_len)
    except ValueError as e:   # still join the all_gather: every rank raises together below
        err, hdr, rec = e, 0, -1
    dev = frame.device
    sizes = torch.tensor([rec], dtype=torch.int64, device=dev)
    all_sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(all_sizes, sizes, group=group)
    lens = [int(s.item()) for s in all_sizes]
    if min(lens) < 0:
        if err is not None:
            raise err
        raise ValueError(f"gather_frame: rank {lens.index(min(lens))} holds no valid -Sx shard frame")
    peer = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
    staged = _host_staged(group, dev)   # gloo: device bytes through pinned host copies
    if rank == dst:
        out = torch.empty(hdr + sum(lens) + 4, dtype=torch.uint8, device=dev)
        ops, pos, mine, land = [], hdr, None, []
        for r, n in enumerate(lens):
            if r == rank:
                mine = (pos, n)
            elif n:
                buf = torch.empty(n, dtype=torch.uint8, pin_memory=True) if staged else out[pos:pos + n]
                land.append((pos, buf))
                ops.append(dist.P2POp(dist.irecv, buf, peer(r), group))
            pos += n
        # receives first (their kernels then get the GPU before anything
        # launched after this call), then the local pieces, which touch
        # other bytes of `out`
        works = dist.batch_isend_irecv(ops) if ops else []
        out[:hdr] = frame[:hdr]
        if mine and mine[1]:
            out[mine[0]:mine[0] + mine[1]] = frame[hdr:hdr + mine[1]]
        out[pos:pos + 4] = 0
        if async_op and not staged:
            return out, works
        for w in works:
            w.wait()
        if staged:
            for p0, buf in land:
                out[p0:p0 + buf.numel()].copy_(buf)
        return (out, []) if async_op else out
    payload = frame[hdr:hdr + rec].cpu() if staged and rec else frame[hdr:hdr + rec]
    works = dist.batch_isend_irecv([dist.P2POp(dist.isend, payload, peer(dst), group)]) if rec else []
    if staged:
        for w in works:
            w.wait()
        works = []
    if async_op:
        return None, works
    for w in works:
        w.wait()
    return None


def walk_records(frame, block_checksum=None):
    """Host walk of the size words of one -Sx frame (bytes): returns (header length, [(start, end), ...], end).

    Mirrors the block loop of decompress() (src/lz4mt.cpp:685-727): a size
    word of 0 ends the frame; bit 31 marks a raw block; a checksum word
    follows the payload when FLG.4 is set.
    """
    frame = bytes(frame)
    hdr, flg = _frame_layout(frame[:20])
    bck = bool(flg & 0x10) if block_checksum is None else block_checksum
    recs, pos = [], hdr
    while True:
        if pos + 4 > len(frame):
            raise ValueError("truncated frame (no EOS)")
        w = struct.unpack_from("<I", frame, pos)[0]
        if w == 0:
            return hdr, recs, pos + 4
        end = pos + 4 + (w & 0x7FFFFFFF) + (4 if bck else 0)
        if end > len(frame):
            raise ValueError("truncated block record")
        recs.append((pos, end))
        pos = end


def split_frame(frame, world):
    """Splits one -Sx frame (bytes) into ``world`` frames of contiguous whole records.

    Each piece is a valid frame (same header, its records, EOS) that decodes
    to the matching slice of the original content; piece r holds the block
    range ``shard_blocks`` assigns to rank r.  This is the host side of the
    decompress scatter.
    """
    frame = bytes(frame)
    hdr, recs, _ = walk_records(frame)
    head = frame[:hdr]
    nb = len(recs)
    out = []
    for r in range(world):
        per, rem = divmod(nb, world)
        first = r * per + min(r, rem)
        count = per + (1 if r < rem else 0)
        body = frame[recs[first][0]:recs[first + count - 1][1]] if count else b""
        out.append(head + body + EOS)
    return out


def rank_blocks(nb, world, rank):
    """(first block, block count) of ``rank`` when nb blocks are split as in ``shard_blocks``."""
    per, rem = divmod(nb, world)
    return rank * per + min(rank, rem), per + (1 if rank < rem else 0)


def host_records(frame, frame_len=None):
    """(header length, [record start offsets..., EOS offset]) of one -Sx frame by a host walk (CPU tensors, bytes)."""
    b = frame[:frame_len].numpy().tobytes() if isinstance(frame, torch.Tensor) else bytes(frame[:frame_len])
    hdr, recs, end = walk_records(b)
    return hdr, [a for a, _ in recs] + [end - 4]


def device_records(frame, frame_len=None):
    """The same from the device walk (lz4mtHipFrameRecords) for a frame in HBM."""
    import lz4mt_amd as L
    hdr, starts, _ = L.frame_records(frame, frame_len)
    return hdr, starts


def _host_staged(group, dev):
    """gloo moves a CUDA tensor by reading it through the host's mapping of
    device memory, ~24 MB/s here (profiles/r04_scatter_split.json): stage
    such transfers through pinned host buffers instead."""
    return dev.type == "cuda" and dist.get_backend(group) == "gloo"


def scatter_frame(frame, frame_len, src=0, group=None, records=None, async_op=False, device=None, stats=None):
    """Cuts ONE -Sx frame held by ``src`` into per-rank sub-frames of whole
    records and delivers piece r to rank r (the decompress side of SURVEY.md
    §8(e): blocks are independent, src/lz4mt.cpp:914-918,991-995).

    ``frame`` is the uint8 tensor on ``src`` (None elsewhere; ``device``: where
    the other ranks receive, default CUDA under RCCL, CPU otherwise); ``records``
    maps (frame, frame_len) to (header length, record starts + EOS offset):
    default the device walk for device tensors, the host walk otherwise.
    Rank r receives blocks ``rank_blocks(nb, world, r)`` as a valid frame
    (the source header, its records, EOS) -- the same split ``shard_blocks``
    makes of the content.  Exchange: one broadcast of the cut table
    (header + 2 x u64 per rank), then grouped sends root -> peers straight
    into each peer's buffer (under gloo, device pieces travel through pinned
    host copies).  Returns the piece (and the works with ``async_op``; host-
    staged transfers are complete on return).  ``stats`` (dict), if given,
    receives the host seconds of the walk, the table broadcast, the
    point-to-point transfers and the piece assembly.
    """
    import time
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    peer = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
    err = None
    t0 = time.perf_counter()
    if rank == src:
        dev = frame.device
        table = torch.zeros(4 + 2 * world, dtype=torch.int64)
        try:
            recs_fn = records or (device_records if frame.is_cuda else host_records)
            hdr, starts = recs_fn(frame, frame_len)
            _frame_layout(bytes(frame[:hdr].cpu().numpy().tobytes()) + b"\0" * 8)
            nb = len(starts) - 1
            table[0] = hdr
            table[1:4] = torch.frombuffer(bytearray(frame[:hdr].cpu().numpy().tobytes().ljust(24, b"\0")),
                                          dtype=torch.int64)
            for r in range(world):
                first, count = rank_blocks(nb, world, r)
                table[4 + 2 * r] = starts[first]
                table[5 + 2 * r] = starts[first + count] - starts[first]
        except Exception as e:   # every rank must leave the broadcast below: flag the error in the table
            err = e
            table.zero_()
            table[0] = -1
        table = table.to(dev)
    else:
        if device is not None:   # where this rank decodes (gloo can carry CUDA tensors too)
            dev = torch.device(device)
        else:
            dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" \
                else torch.device("cpu")
        table = torch.zeros(4 + 2 * world, dtype=torch.int64, device=dev)
    t1 = time.perf_counter()
    staged = _host_staged(group, dev)
    if staged:   # the table too: 8 B per rank through gloo's host path
        tb = table.cpu()
        dist.broadcast(tb, peer(src), group=group)
        table = tb
    else:
        dist.broadcast(table, peer(src), group=group)
    if int(table[0].item()) < 0:   # the source rank could not cut the frame: all ranks raise together
        if err is not None:
            raise err
        raise ValueError(f"scatter_frame: rank {src} could not walk the frame")
    t = table.cpu().tolist()
    t2 = time.perf_counter()
    hdr = int(t[0])
    head = torch.tensor(t[1:4], dtype=torch.int64).numpy().tobytes()[:hdr]
    off, ln = int(t[4 + 2 * rank]), int(t[5 + 2 * rank])
    piece = torch.empty(hdr + ln + 4, dtype=torch.uint8, device=dev)
    works, landing = [], None
    if rank == src:
        ops = []
        for r in range(world):
            a, b = int(t[4 + 2 * r]), int(t[5 + 2 * r])
            if r == rank or not b:
                continue
            chunk = frame[a:a + b]
            if staged:
                chunk = chunk.to("cpu", non_blocking=False)
            ops.append(dist.P2POp(dist.isend, chunk, peer(r), group))
        works = dist.batch_isend_irecv(ops) if ops else []
    elif ln:
        landing = torch.empty(ln, dtype=torch.uint8, pin_memory=True) if staged else piece[hdr:hdr + ln]
        works = dist.batch_isend_irecv([dist.P2POp(dist.irecv, landing, peer(src), group)])
    if staged or not async_op:
        for w in works:
            w.wait()
        works = []
    t3 = time.perf_counter()
    if rank == src and ln:
        piece[hdr:hdr + ln] = frame[off:off + ln]
    elif staged and ln:
        piece[hdr:hdr + ln].copy_(landing)
    piece[:hdr] = torch.frombuffer(bytearray(head), dtype=torch.uint8).to(dev)
    piece[hdr + ln:] = 0
    if stats is not None:
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        stats.update(walk_s=t1 - t0, table_s=t2 - t1, p2p_s=t3 - t2, assemble_s=time.perf_counter() - t3,
                     host_staged=staged, piece_bytes=piece.numel())
    if async_op:
        return piece, works
    return piece


def _all_gather_var(t, group=None):
    """all_gather of 1-D int64 tensors whose lengths differ by rank."""
    world = dist.get_world_size(group)
    n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
    ns = [torch.zeros(1, dtype=torch.int64, device=t.device) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    lens = [int(x.item()) for x in ns]
    m = max(lens + [1])
    pad = torch.zeros(m, dtype=torch.int64, device=t.device)
    pad[:t.numel()] = t
    bufs = [torch.zeros(m, dtype=torch.int64, device=t.device) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return [b[:k] for b, k in zip(bufs, lens)]


def verify_stitched(full, shard_src, decode, digests, dst=0, group=None, records=None):
    """Checks a stitched frame (on ``dst``) against every rank's source shard.

    Every rank passes its source ``shard_src`` (uint8 tensor); ``digests``
    maps a uint8 tensor to an int64 tensor of chunk digests (e.g. XXH32 of
    16 MiB pieces, lz4mtHipXxh32Chunks); ``decode`` maps a frame to its
    content (root only).  The root walks the stitched frame's size words
    (``records``: default the device walk for device tensors, the host walk
    otherwise), cuts it at each shard's block range and decodes the pieces
    one at a time (header + that shard's records + EOS: valid frames,
    src/lz4mt.cpp:914-918), comparing each piece's content digests with the
    all-gathered ones.  So the root holds one shard's content at a time, not
    the whole stream's (64 GiB at configs[3]).  Returns True on every rank
    iff every shard matches and the frame holds exactly their blocks.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    mine = digests(shard_src).to(torch.int64)
    sizes = _all_gather_var(torch.tensor([shard_src.numel()], dtype=torch.int64, device=mine.device), group)
    allsum = _all_gather_var(mine, group)
    ok = torch.ones(1, dtype=torch.int64, device=mine.device)
    err = None
    if rank == dst:
        try:
            recs_fn = records or (device_records if full.is_cuda else host_records)
            hdr, starts = recs_fn(full, full.numel())
            head = full[:hdr]
            bd = int(head[5].item())
            bm = block_bytes((bd >> 4) & 7)
            counts = [(int(sizes[r].item()) + bm - 1) // bm for r in range(world)]
            good = sum(counts) == len(starts) - 1
            first = 0
            for r in range(world):
                if not good:
                    break
                n = int(sizes[r].item())
                body = full[starts[first]:starts[first + counts[r]]]
                first += counts[r]
                piece = torch.cat([head, body, torch.zeros(4, dtype=torch.uint8, device=full.device)])
                del body
                out = decode(piece)
                del piece
                if out.numel() != n or not torch.equal(digests(out).to(torch.int64).cpu(), allsum[r].cpu()):
                    good = False
                del out
            ok[0] = 1 if good else 0
        except Exception as e:   # still reach the broadcast, so no rank waits forever
            err = e
            ok[0] = -1
    peer = dist.get_global_rank(group, dst) if group is not None else dst
    dist.broadcast(ok, peer, group=group)
    v = int(ok.item())
    if v < 0:
        if err is not None:
            raise err
        raise RuntimeError(f"verify_stitched: rank {dst} could not decode the stitched frame")
    return v == 1


# ---------------------------------------------------------------------------
# Streamed gather: the compress-side exchange overlapped with the encode
# ---------------------------------------------------------------------------
PACK_HDR = 64   # lz4mtHipShardPack's header: u64 magic, payload, remaining, pack bytes; u32 nb, flags; u64 body


def parse_pack_header(b):
    """(pack bytes, payload bytes, shard complete, the shard's record bytes) from a pack header (64 bytes)."""
    magic, payload, _remaining, packed, _nb, flags, body = struct.unpack_from("<QQQQIIQ", bytes(b), 0)
    if magic != 0x44485354344D5A4C:
        raise ValueError("not a shard pack")
    return packed, payload, bool(flags & 1), body


class HipShardEngine:
    """The device side of compress_gather_streamed on this rank's GPU
    (include/lz4mt_hip.h section 4).  The encode runs on its own stream and
    the rounds' packs on another, so that neither the encode nor the RCCL
    transfers (which torch orders after the CURRENT stream) wait for each
    other."""

    def __init__(self, device=None):
        import lz4mt_amd as L
        self.L = L
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.enc_stream = torch.cuda.Stream(self.device)
        self.pack_stream = torch.cuda.Stream(self.device)
        self.enc_done = torch.cuda.Event()

    def header(self, sd):
        return self.L.frame_header(sd)

    def workspace(self, n, sd):
        return self.L.shard_workspace(n, sd, device=self.device)

    def pack_buffer(self, n, sd, cap):
        return torch.empty(self.L.shard_pack_bound(n, sd, cap), dtype=torch.uint8, device=self.device)

    def encode(self, src, sd, ws):
        # the round state is zeroed on the CURRENT stream, which both the
        # encode stream (here) and the pack stream (every pack) wait on: no
        # pack can read `sent` / `pub` before the reset, and no reset can
        # land after a pack wrote them
        self.L.shard_reset(src.numel(), sd, ws, stream=torch.cuda.current_stream(self.device))
        self.enc_stream.wait_stream(torch.cuda.current_stream(self.device))   # src / ws ready, ws reset
        self.enc_start = torch.cuda.Event(enable_timing=True)
        self.enc_done = torch.cuda.Event(enable_timing=True)
        self.enc_start.record(self.enc_stream)
        self.L.shard_encode(src, sd, ws, stream=self.enc_stream)
        self.enc_done.record(self.enc_stream)

    def encode_finished(self):
        return self.enc_done.query()

    def pack(self, src, sd, ws, buf, cap, final):
        """One round; returns parse_pack_header's fields -- waits for the pack."""
        ps = self.pack_stream
        ps.wait_stream(torch.cuda.current_stream(self.device))   # the previous send of `buf` is done
        if final:
            ps.wait_event(self.enc_done)
        self.L.shard_pack(src, sd, ws, buf, cap, final, stream=ps)
        with torch.cuda.stream(ps):
            h = buf[:PACK_HDR].cpu()   # synchronises the pack stream
        return parse_pack_header(h.numpy().tobytes())

    def unpack(self, buf, n, sd, mirror):
        self.L.shard_unpack(buf, n, sd, mirror)

    def body_bytes(self, n, sd, ws):
        torch.cuda.current_stream(self.device).wait_event(self.enc_done)
        return self.L.shard_body_bytes(n, sd, ws)

    def assemble(self, src, n, sd, ws, body):
        torch.cuda.current_stream(self.device).wait_event(self.enc_done)
        self.L.shard_assemble(src, n, sd, ws, body)


class RcclTransport:
    """Packs travel as point-to-point transfers of a torch.distributed group
    (RCCL under the nccl backend) after each round's exchange of sizes.  On
    MI355X an RCCL transfer is a kernel needing ~37 KiB of LDS per
    workgroup, which no CU has free while its 8 encoder waves hold all 160
    KiB: the transfers then wait for the encodes to end.  Used by the CPU
    tests (gloo) and as the fallback of IpcPushTransport."""

    def __init__(self, group=None):
        self.group = group

    def setup(self, E, sizes, sd, cap, rank, dst, ctrl):
        self.rank, self.dst = rank, dst
        self.recv = {r: E.pack_buffer(sizes[r], sd, cap) for r in range(len(sizes)) if r != dst} \
            if rank == dst else {}

    def push(self, k, buf, nbytes):
        pass

    def exchange(self, k, buf, rows):
        peer = (lambda r: dist.get_global_rank(self.group, r)) if self.group is not None else (lambda r: r)
        ops = []
        if self.rank == self.dst:
            for r, row in enumerate(rows):
                if r != self.dst and row[0]:
                    ops.append(dist.P2POp(dist.irecv, self.recv[r][:row[0]], peer(r), self.group))
        elif rows[self.rank][0]:
            ops.append(dist.P2POp(dist.isend, buf[:rows[self.rank][0]], peer(self.dst), self.group))
        for w in (dist.batch_isend_irecv(ops) if ops else []):
            w.wait()

    def received(self, r, k):
        return self.recv[r]

    def close(self):
        self.recv = {}


class IpcSetupError(RuntimeError):
    """IpcPushTransport.setup failed on some rank; raised on EVERY rank (the
    setup is collective), so the caller may fall back to another transport
    together.  Any other error inside the rounds is not collective and must
    end the process."""


def peer_access_matrix():
    """hipDeviceCanAccessPeer for every ordered pair of visible devices
    (list of rows; True on the diagonal)."""
    n = torch.cuda.device_count()
    return [[i == j or bool(torch.cuda.can_device_access_peer(i, j)) for j in range(n)] for i in range(n)]


def dist_timeout():
    """Timeout of every process group this path makes (init_process_group in
    bench.py, the gloo control group): a rank that stops answering ends the
    run with an error instead of stalling it for torch's default 30 min.
    LZ4MT_DIST_TIMEOUT_S overrides the 300 s default."""
    import datetime
    import os
    return datetime.timedelta(seconds=float(os.environ.get("LZ4MT_DIST_TIMEOUT_S", "300")))


def _bus_id(L, dev_index):
    buf = ctypes.create_string_buffer(64)
    return buf.value.decode() if L.lib.lz4mtHipDevicePciBusId(int(dev_index), buf, 64) == 0 else None


class IpcPushTransport:
    """Each sender's pack goes straight into a receive buffer in the root's
    HBM, exported once by IPC handle (lz4mtHipIpcAllocKind / lz4mtHipIpcOpen),
    with an asynchronous device-to-device copy (lz4mtHipCopyAsync: a copy
    engine over xGMI, no kernel and no LDS) before the round's exchange; two
    buffers per sender alternate, and the root finishes unpacking round k
    before it joins round k + 1's exchange, so a sender never overwrites a
    pack the root still reads.  Only the round's sizes go over the (gloo)
    control group.

    Visibility on the root: a peer's copy-engine writes land in the root's
    HBM behind the back of its XCD L2s.  The receive buffers are uncached
    device memory (no L2 line of them is ever held); a runtime that cannot
    export uncached memory by IPC fails the setup (IpcSetupError -> RCCL),
    since a cached buffer could serve stale lines of an earlier round that
    no set-up check can provoke.  The root's k_shard_unpack
    also starts every workgroup with a system-scope acquire (buffer_inv sc0
    sc1).  The setup then PROVES the path end to end: every
    sender pushes a seeded pattern into both of its buffers and the root
    compares the XXH32 of every 1 MiB piece with the sender's; any mismatch
    (or a failed map / peer-access check) raises IpcSetupError on every rank
    together, and the caller falls back to RcclTransport.  The root's GPU is
    named by PCI bus id, which each sender resolves to its own ordinal, so
    ranks that number devices differently still agree.

    The buffers are kept for the next call with the same layout (shard
    sizes, descriptor, per-block cap, root); a call with another layout
    tears them down and sets up again, on every rank alike (every rank sees
    the same all-gathered layout)."""

    CHUNK = 1 << 20   # pattern check granule

    def __init__(self, device):
        self.device = device
        self.bufs, self.remote, self.copy_stream = {}, [], None
        self.key, self.cap_bytes, self.kind = None, 0, None

    @staticmethod
    def _layout_key(sizes, sd, cap, dst):
        return (tuple(sizes), bytes(sd), int(cap), int(dst))

    def setup(self, E, sizes, sd, cap, rank, dst, ctrl):
        """Collective over ``ctrl``: every rank either sets up (and passes the
        pattern check) or raises IpcSetupError."""
        import lz4mt_amd as L
        key = self._layout_key(sizes, sd, cap, dst)
        if (self.bufs or self.remote) and key == self.key:   # an earlier call with this same layout
            return
        if self.bufs or self.remote:   # another layout: every rank sees the same sizes, so all re-set up
            self.close()
        self.L, self.rank, self.dst = L, rank, dst
        me = self.device.index if self.device.index is not None else torch.cuda.current_device()
        handles, kinds, err = {}, [], None
        if rank == dst:
            try:
                for r in range(len(sizes)):
                    if r == dst:
                        continue
                    nbytes = L.shard_pack_bound(sizes[r], sd, cap)
                    pair = []
                    self.bufs[r] = pair
                    for _ in range(2):
                        ptr, h, k = ctypes.c_void_p(), (ctypes.c_uint8 * 64)(), ctypes.c_int(-1)
                        if L.lib.lz4mtHipIpcAllocKind(nbytes, ctypes.byref(ptr), h, 2, ctypes.byref(k)) != 0:
                            raise IpcSetupError("lz4mtHipIpcAllocKind failed")
                        pair.append(ptr.value)
                        kinds.append(k.value)
                        handles.setdefault(r, []).append(bytes(h))
                        if k.value != 2:
                            # a cached (fine- or coarse-grained)
                            # receive buffer can hold L2 lines from the root's
                            # unpack two rounds back, which a system-scope
                            # acquire does not drop for coarse-grained memory
                            # on gfx942/950, and the set-up pattern check runs
                            # before any such line exists -- so it cannot prove
                            # those kinds; only uncached memory is taken
                            raise IpcSetupError(f"the runtime exported no uncached receive buffer (got kind "
                                                f"{k.value}); cached kinds are not used for the IPC push")
            except IpcSetupError as e:
                err, handles = e, None
        obj = [handles, _bus_id(L, me) if rank == dst else None, min(kinds) if kinds else None]
        dist.broadcast_object_list(obj, src=dst if ctrl is None else dist.get_global_rank(ctrl, dst), group=ctrl)
        ok = obj[0] is not None
        names = {2: "uncached", 1: "fine-grained", 0: "coarse-grained"}
        self.kind = names.get(obj[2], "none")
        if ok and rank != dst:
            try:
                rd = L.lib.lz4mtHipDeviceByPciBusId(obj[1].encode()) if obj[1] else -1
                # rd < 0: the root's GPU is not visible to this process (its
                # own device list is restricted); the map and the pattern
                # check below still decide
                if rd >= 0 and rd != me and L.lib.lz4mtHipCanAccessPeer(me, rd) != 1:
                    raise IpcSetupError(f"device {me} cannot access the root's device {rd} = {obj[1]} "
                                        "(hipDeviceCanAccessPeer)")
                self.cap_bytes = L.shard_pack_bound(sizes[rank], sd, cap)
                for h in obj[0][rank]:
                    ptr = ctypes.c_void_p()
                    hb = (ctypes.c_uint8 * 64).from_buffer_copy(h)
                    if L.lib.lz4mtHipIpcOpen(hb, ctypes.byref(ptr)) != 0:
                        raise IpcSetupError("lz4mtHipIpcOpen failed")
                    self.remote.append(ptr.value)
                self.copy_stream = torch.cuda.Stream(self.device)
            except IpcSetupError as e:
                err, ok = e, False
        if self._all_ok(ok, ctrl):
            ok, err = self._pattern_check(sizes, sd, cap, ctrl)
            if self._all_ok(ok, ctrl):
                self.key = key
                return
        self.close()
        raise err or IpcSetupError("IpcPushTransport: another rank failed the setup or the pattern check")

    @staticmethod
    def _all_ok(ok, ctrl):
        flag = torch.tensor([1 if ok else 0], dtype=torch.int64)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=ctrl)
        return int(flag.item()) == 1

    def _pattern_check(self, sizes, sd, cap, ctrl):
        """Every sender fills both of its root buffers with a seeded pattern
        (through the same copies the rounds use); the root hashes what
        arrived, 1 MiB at a time, and compares.  Returns (ok, error) on every
        rank.  LZ4MT_AMD_IPC_CORRUPT=1 (tests) flips one pattern byte after
        the sender's digests are taken, so the check must fail."""
        import os
        L = self.L
        digs = None
        if self.rank != self.dst:
            n = self.cap_bytes
            g = torch.Generator(device=self.device)
            g.manual_seed(0x5EED + 7919 * self.rank)
            digs = []
            st = self.copy_stream
            for k in range(2):
                pat = torch.randint(0, 256, (n,), dtype=torch.uint8, device=self.device, generator=g)
                digs.append(L.xxh32_chunks(pat, self.CHUNK).cpu().tolist())
                if os.environ.get("LZ4MT_AMD_IPC_CORRUPT") == "1":
                    pat[n // 2] ^= 0x5A
                st.wait_stream(torch.cuda.current_stream(self.device))
                if L.lib.lz4mtHipCopyAsync(ctypes.c_void_p(self.remote[k]), ctypes.c_void_p(pat.data_ptr()), n,
                                           ctypes.c_void_p(st.cuda_stream)) != 0:
                    return False, IpcSetupError("lz4mtHipCopyAsync failed during the pattern check")
                st.synchronize()
                del pat
        world = dist.get_world_size(ctrl)
        alld = [None] * world
        dist.all_gather_object(alld, digs, group=ctrl)
        if self.rank != self.dst:
            return True, None
        bad = []
        cur = torch.cuda.current_stream(self.device)
        for r, pair in self.bufs.items():
            n = L.shard_pack_bound(sizes[r], sd, cap)
            nc = (n + self.CHUNK - 1) // self.CHUNK
            for k, ptr in enumerate(pair):
                out = torch.empty(nc, dtype=torch.int32, device=self.device)
                if L.lib.lz4mtHipXxh32Chunks(ctypes.c_void_p(ptr), n, self.CHUNK, ctypes.c_void_p(out.data_ptr()),
                                             ctypes.c_void_p(cur.cuda_stream)) != 0:
                    return False, IpcSetupError("lz4mtHipXxh32Chunks failed during the pattern check")
                got = [v & 0xFFFFFFFF for v in out.cpu().tolist()]
                want = [v & 0xFFFFFFFF for v in (alld[r][k] if alld[r] else [])]
                if got != want:
                    bad.append((r, k))
        if bad:
            return False, IpcSetupError(f"IPC pattern check failed: (sender, buffer) {bad} did not arrive intact "
                                        f"in the root's {self.kind} receive buffers")
        return True, None

    def push(self, k, buf, nbytes):
        if self.rank == self.dst or not nbytes:
            if self.rank == self.dst:   # round k - 1's unpacks are done before round k's exchange
                torch.cuda.current_stream(self.device).synchronize()
            return
        if nbytes > self.cap_bytes or nbytes > buf.numel():   # never write past the root's buffer
            raise RuntimeError(f"IpcPushTransport: pack of {nbytes} B exceeds the root buffer ({self.cap_bytes} B)")
        st = self.copy_stream
        if self.L.lib.lz4mtHipCopyAsync(ctypes.c_void_p(self.remote[k % 2]), ctypes.c_void_p(buf.data_ptr()), nbytes,
                                        ctypes.c_void_p(st.cuda_stream)) != 0:
            raise RuntimeError("lz4mtHipCopyAsync failed")
        st.synchronize()

    def exchange(self, k, buf, rows):
        pass

    def received(self, r, k):
        return self.bufs[r][k % 2]

    def close(self):
        for p in self.remote:
            self.L.lib.lz4mtHipIpcClose(ctypes.c_void_p(p))
        for pair in self.bufs.values():
            for p in pair:
                self.L.lib.lz4mtHipFree(ctypes.c_void_p(p))
        self.bufs, self.remote, self.key, self.cap_bytes = {}, [], None, 0


_CTRL_GROUPS = {}


def control_group(group=None):
    """A gloo group over the ranks of ``group`` for the rounds' size
    exchange (CPU tensors, no GPU kernel); ``group`` itself when it already
    is gloo.  Made once per group (collective on first use)."""
    if dist.get_backend(group) == "gloo":
        return group
    # keyed by the group AND the default group, compared by identity (an id()
    # of a destroyed group can be reused by a new one), so a new
    # process group in the same process gets a new control group
    world = dist.group.WORLD
    key = id(group) if group is not None else None
    hit = _CTRL_GROUPS.get(key)
    if hit is None or hit[0] is not group or hit[1] is not world:
        ranks = dist.get_process_group_ranks(group) if group is not None else None
        _CTRL_GROUPS[key] = (group, world, dist.new_group(ranks=ranks, backend="gloo", timeout=dist_timeout()))
    return _CTRL_GROUPS[key][2]


def _shard_sizes(n, world, ctrl):
    alln = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(alln, torch.tensor([n], dtype=torch.int64), group=ctrl)
    return [int(x.item()) for x in alln]


def prepare_transport(transport, engine, n, sd, dst=0, group=None, ctrl=None, per_block_cap=128 << 10):
    """Sets ``transport`` up for compress_gather_streamed calls over shards of
    this layout (this rank's shard: n bytes), collectively, ahead of any
    timed call: the IPC buffers, their export, the senders' maps and the
    pattern check happen here instead of inside the first call.  Raises
    IpcSetupError on every rank together when the IPC path is not usable."""
    ctrl = ctrl if ctrl is not None else control_group(group)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    transport.setup(engine, _shard_sizes(n, world, ctrl), sd, per_block_cap, rank, dst, ctrl)


def compress_gather_streamed(src, sd, dst=0, group=None, engine=None, per_block_cap=128 << 10, ws=None, stats=None,
                             min_round_s=0.002, transport=None, ctrl=None):
    """Compresses this rank's shard and gathers every shard's records into ONE
    frame on ``dst`` WHILE the shards encode.

    Each rank holds a contiguous block range of one stream (ranks in stream
    order, ``shard_blocks``), ``src`` its bytes.  Every rank launches its
    encode (lz4mtHipShardEncode: 1 and 4 MiB blocks publish their progress
    every 64 KiB of output), then the ranks run rounds together until every
    shard is complete: a sender packs what its encoder has published since
    the last round (at most ``per_block_cap`` bytes per block; after its
    encode: the tails, incompressible blocks' source bytes, stored sizes and
    block checksums) and hands it to the ``transport`` (IpcPushTransport: a
    copy-engine write into the root's buffer; RcclTransport, the default:
    point-to-point after the exchange); one all_gather over ``ctrl`` (a gloo
    group: no GPU kernel) of (pack bytes, complete, record bytes) per rank;
    the root unpacks each pack into its mirror of that shard.  At the end the
    root assembles each shard's records at its place in the frame (header,
    records in rank order, EOS): byte for byte the frame one process writes
    for the whole stream (src/lz4mt.cpp:898-935; blocks are independent,
    914-918).  Returns the frame on ``dst`` (None elsewhere).  ``stats``
    (dict), if given, receives the round count and the bytes per round.
    While the encodes run, rounds start at least ``min_round_s`` apart.
    """
    import time
    ctrl = ctrl if ctrl is not None else control_group(group)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    E = engine or HipShardEngine(src.device)
    T = transport or RcclTransport(group)
    dev = src.device
    n = src.numel()
    sizes = _shard_sizes(n, world, ctrl)
    # the stitched frame is the whole stream's only if every shard but the
    # last non-empty one is a whole number of blocks (every rank sees the
    # same sizes, so every rank raises here together)
    bm = block_bytes(sd.bd.blockMaximumSize)
    last = max([r for r in range(world) if sizes[r]] or [0])
    bad = [r for r in range(last) if sizes[r] % bm]
    if bad:
        raise ValueError(f"compress_gather_streamed: shard(s) {bad} are not whole {bm}-byte blocks "
                         "and are followed by another shard (use shard_blocks)")
    ws = ws if ws is not None else E.workspace(n, sd)
    T.setup(E, sizes, sd, per_block_cap, rank, dst, ctrl)
    E.encode(src, sd, ws)
    mirrors = {r: E.workspace(sizes[r], sd) for r in range(world) if r != rank} if rank == dst else {}
    bufs = [] if rank == dst else [E.pack_buffer(n, sd, per_block_cap), E.pack_buffer(n, sd, per_block_cap)]
    complete = rank == dst          # the root sends nothing; it assembles its own shard from its workspace
    body = {}
    rounds, sent_log = 0, []
    t_last = 0.0
    t_start = time.perf_counter()
    t_final = None          # when this rank first found its encode finished
    rounds_after = 0        # rounds from then on (the tail)
    while True:
        nbytes, body_now, now_complete = 0, 0, complete
        buf = None
        if not complete:
            final = E.encode_finished()
            if final and t_final is None:
                t_final = time.perf_counter()
            if not final:
                wait = t_last + min_round_s - time.perf_counter()
                if wait > 0:
                    time.sleep(wait)
            t_last = time.perf_counter()
            buf = bufs[rounds % 2]
            nbytes, payload, done, b = E.pack(src, sd, ws, buf, per_block_cap, final)
            if final and done:
                now_complete, body_now = True, b
            elif not payload:
                nbytes = 0   # nothing published since the last round: send nothing
        T.push(rounds, buf, nbytes)
        info = torch.tensor([nbytes, 1 if now_complete else 0, body_now], dtype=torch.int64)
        alli = [torch.zeros(3, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(alli, info, group=ctrl)
        rows = [[int(v) for v in x.tolist()] for x in alli]
        T.exchange(rounds, buf, rows)
        if rank == dst:
            for r in range(world):
                if r != rank and rows[r][0]:
                    E.unpack(T.received(r, rounds), sizes[r], sd, mirrors[r])
        for r in range(world):
            if rows[r][1] and r not in body:
                body[r] = rows[r][2]
        complete = now_complete
        rounds += 1
        if t_final is not None:
            rounds_after += 1
        sent_log.append(sum(row[0] for row in rows))
        if all(row[1] for row in rows):
            break
    t_rounds = time.perf_counter()
    if stats is not None:
        stats.update(rounds=rounds, bytes_per_round=sent_log, rounds_after_encode=rounds_after,
                     loop_s=t_rounds - t_start,
                     tail_rounds_s=(t_rounds - t_final) if t_final is not None else None)
    if rank != dst:
        return None
    body[rank] = E.body_bytes(n, sd, ws)
    if stats is not None:
        stats["own_body_bytes"] = body[rank]
    head = E.header(sd)
    total = len(head) + sum(body[r] for r in range(world)) + 4
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    out[:len(head)] = torch.frombuffer(bytearray(head), dtype=torch.uint8).to(dev)
    pos = len(head)
    for r in range(world):
        piece = out[pos:pos + body[r]]
        if r == rank:
            E.assemble(src, n, sd, ws, piece)
        else:
            E.assemble(None, sizes[r], sd, mirrors[r], piece)
        pos += body[r]
    out[pos:pos + 4] = 0
    if stats is not None:   # host time of the root's own-size readback + assembly launches (not synchronised)
        stats["assemble_launch_s"] = time.perf_counter() - t_rounds
    return out
