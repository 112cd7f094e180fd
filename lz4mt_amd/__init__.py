"""lz4mt_amd — MI355X-native LZ4 frame codec behind the t-mat/lz4mt API.

The product is the C-ABI library ``liblz4mt_amd.so`` (HIP kernels for gfx950
+ the C++ frame engine).  This package is the Python host mirror of the
reference's interface (src/lz4mt.h): ``init_context``,
``init_stream_descriptor``, ``compress`` / ``decompress`` over callbacks,
plus device-resident helpers that take torch tensors (torch supplies device
memory and streams only).

torch is imported before the library is loaded so that both bind the same
libamdhip64 (identical soname); there is no CPU fallback: on a machine
without a HIP device every compute entry point returns an error.
"""
import ctypes
import weakref

import torch  # noqa: F401  (must precede the CDLL load: shared HIP runtime)

from . import _abi
from ._abi import (MODE_DEVICE, MODE_PARALLEL, MODE_SEQUENTIAL, RESULT_NAMES, Lz4MtContext, Lz4MtMemIo,
                   Lz4MtStreamDescriptor, Result)

__all__ = [
    "lib", "Result", "RESULT_NAMES", "MODE_PARALLEL", "MODE_SEQUENTIAL", "MODE_DEVICE", "Lz4MtError",
    "init_context", "init_stream_descriptor", "result_to_string", "result_to_exit_code", "make_sd",
    "compress", "decompress", "compress_block", "decompress_block", "compress_bound",
    "compress_frame", "decompress_frame", "frame_info", "frame_bound", "gen_synthetic", "xxh32",
    "device_count", "stream_bound", "frame_records", "xxh32_chunks", "frame_header", "shard_workspace",
    "shard_pack_bound", "shard_reset", "shard_encode", "shard_pack", "shard_unpack", "shard_assemble", "shard_body_bytes",
]

lib = _abi.load()


class Lz4MtError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = int(code)
        name = RESULT_NAMES[code] if 0 <= code < len(RESULT_NAMES) else result_to_string(code)
        super().__init__(f"{what}: {name} ({code})")


def init_context():
    """lz4mtInitContext (reference src/lz4mt.cpp:851-871)."""
    return lib.lz4mtInitContext()


def init_stream_descriptor():
    """lz4mtInitStreamDescriptor (reference src/lz4mt.cpp:874-895)."""
    return lib.lz4mtInitStreamDescriptor()


def result_to_string(code):
    return lib.lz4mtResultToString(int(code)).decode()


def result_to_exit_code(code):
    return lib.lz4mtResultToLz4cExitCode(int(code))


def make_sd(block_max_id=7, stream_checksum=True, block_checksum=False, stream_size=None, block_dependence=False):
    """Stream descriptor with the CLI's flag mapping (-B#, -BX, -BD, -Sx)."""
    sd = init_stream_descriptor()
    sd.bd.blockMaximumSize = block_max_id
    sd.flg.blockIndependence = 0 if block_dependence else 1
    sd.flg.streamChecksum = 1 if stream_checksum else 0
    sd.flg.blockChecksum = 1 if block_checksum else 0
    if stream_size is not None:
        sd.flg.streamSize = 1
        sd.streamSize = int(stream_size)
    return sd


def device_count():
    return lib.lz4mtHipDeviceCount()


# ---------------------------------------------------------------------------
# callback API over memory buffers (lz4mtCompress / lz4mtDecompress)
# ---------------------------------------------------------------------------
def _run(fn, data, sd, mode, level, out_cap, compress_cb=None, decompress_cb=None):
    src = ctypes.create_string_buffer(bytes(data), len(data) or 1)
    out = ctypes.create_string_buffer(max(out_cap, 1))
    io = Lz4MtMemIo(ctypes.cast(src, ctypes.c_void_p), len(data), 0, 0, ctypes.cast(out, ctypes.c_void_p),
                    out_cap, 0)
    ctx = init_context()
    ctx.mode = mode
    ctx.compressionLevel = level
    lib.lz4mtMemBind(ctypes.byref(ctx), ctypes.byref(io))
    keep = []
    if compress_cb is not None:
        keep.append(_abi.COMPRESS_FN(compress_cb))
        ctx.compress = ctypes.cast(keep[-1], ctypes.c_void_p)
    if decompress_cb is not None:
        keep.append(_abi.DECOMPRESS_FN(decompress_cb))
        ctx.decompress = ctypes.cast(keep[-1], ctypes.c_void_p)
    r = fn(ctypes.byref(ctx), ctypes.byref(sd))
    return r, out.raw[:io.outPos]


def compress(data, sd=None, mode=MODE_PARALLEL, level=0, compress_cb=None):
    """Frame-compresses ``data`` through lz4mtCompress; returns (result, frame bytes).

    Null codec callbacks run every block on the GPU (lz4mtHipCompressBlock);
    ``mode=MODE_DEVICE`` uses the batched device engine.
    """
    sd = sd if sd is not None else init_stream_descriptor()
    bm = 1 << (8 + 2 * sd.bd.blockMaximumSize) if 4 <= sd.bd.blockMaximumSize <= 7 else 4 << 20
    cap = 64 + len(data) + 8 * (len(data) // bm + 2)
    return _run(lib.lz4mtCompress, data, sd, mode, level, cap, compress_cb=compress_cb)


def decompress(frame, out_cap, mode=MODE_PARALLEL, decompress_cb=None):
    """lz4mtDecompress over memory; returns (result, decoded bytes, last stream descriptor)."""
    sd = init_stream_descriptor()
    r, out = _run(lib.lz4mtDecompress, frame, sd, mode, 0, out_cap, decompress_cb=decompress_cb)
    return r, out, sd


# ---------------------------------------------------------------------------
# block operators (reference plugin signatures, host memory)
# ---------------------------------------------------------------------------
def compress_bound(n):
    return lib.lz4mtHipCompressBound(int(n))


def compress_block(data, cap=None, level=0):
    """lz4mtHipCompressBlock: LZ4_compress_limitedOutput semantics; returns bytes (b'' if it does not fit)."""
    data = bytes(data)
    cap = len(data) if cap is None else int(cap)
    dst = ctypes.create_string_buffer(max(cap, compress_bound(len(data))) + 16)
    n = lib.lz4mtHipCompressBlock(data, dst, len(data), cap, level)
    if n < 0:
        raise Lz4MtError(Result.ERROR, "lz4mtHipCompressBlock")
    return dst.raw[:n]


def decompress_block(block, cap):
    """lz4mtHipDecompressBlock: returns (ret, bytes) with ret < 0 for malformed input."""
    block = bytes(block)
    dst = ctypes.create_string_buffer(max(int(cap), 1) + 16)
    n = lib.lz4mtHipDecompressBlock(block, dst, len(block), int(cap))
    return n, (dst.raw[:n] if n > 0 else b"")


# ---------------------------------------------------------------------------
# device-resident frame engine (torch uint8 tensors on the current device)
# ---------------------------------------------------------------------------
def _stream(stream):
    if stream is None:
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    return ctypes.c_void_p(stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream))


def _check_dev(t, name):
    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.uint8 and t.is_contiguous()):
        raise TypeError(f"{name} must be a contiguous torch.uint8 tensor on a HIP device")


def frame_bound(n, sd=None):
    sd = sd if sd is not None else init_stream_descriptor()
    return int(lib.lz4mtHipFrameBound(int(n), ctypes.byref(sd)))


def compress_workspace(n, sd=None, device=None, level=0):
    sd = sd if sd is not None else init_stream_descriptor()
    nbytes = int(lib.lz4mtHipCompressWorkspaceSizeEx(int(n), ctypes.byref(sd), int(level)))
    return torch.empty(nbytes, dtype=torch.uint8, device=device or "cuda")


def compress_frame(src, sd=None, out=None, workspace=None, stream=None, level=0):
    """Compresses a device tensor into one lz4mt frame; returns the frame tensor (a view of ``out``).
    ``level`` >= 3 selects LZ4-HC (the reference's codec for those levels:
    3..9 hashChain, 10..12 and above the optimal parser)."""
    _check_dev(src, "src")
    sd = sd if sd is not None else init_stream_descriptor()
    n = src.numel()
    cap = frame_bound(n, sd)
    if out is None:
        out = torch.empty(cap, dtype=torch.uint8, device=src.device)
    fs = ctypes.c_uint64(0)
    ws_ptr, ws_size = (workspace.data_ptr(), workspace.numel()) if workspace is not None else (None, 0)
    r = lib.lz4mtHipCompressFrameEx(ctypes.c_void_p(src.data_ptr() if n else out.data_ptr()), n,
                                    ctypes.c_void_p(out.data_ptr()), out.numel(), ctypes.byref(fs),
                                    ctypes.byref(sd), int(level), ctypes.c_void_p(ws_ptr), ws_size, _stream(stream))
    if r != Result.OK:
        raise Lz4MtError(r, "lz4mtHipCompressFrame")
    return out[:fs.value]


def frame_info(frame, stream=None):
    """(stream descriptor, decoded-size bound, block count) of the first frame."""
    _check_dev(frame, "frame")
    sd = init_stream_descriptor()
    bound, nb = ctypes.c_uint64(0), ctypes.c_uint64(0)
    r = lib.lz4mtHipFrameInfo(ctypes.c_void_p(frame.data_ptr()), frame.numel(), ctypes.byref(sd),
                              ctypes.byref(bound), ctypes.byref(nb), _stream(stream))
    if r != Result.OK:
        raise Lz4MtError(r, "lz4mtHipFrameInfo")
    return sd, bound.value, nb.value


def stream_bound(frame, stream=None):
    """Decoded-size bound of every frame in the device bytes (concatenated and skippable frames included)."""
    _check_dev(frame, "frame")
    b = ctypes.c_uint64(0)
    r = lib.lz4mtHipStreamBound(ctypes.c_void_p(frame.data_ptr()), frame.numel(), ctypes.byref(b), _stream(stream))
    if r != Result.OK:
        raise Lz4MtError(r, "lz4mtHipStreamBound")
    return b.value


def frame_records(frame, frame_len=None, stream=None):
    """(header length, [record start offsets..., EOS offset], descriptor) of one device frame (device walk)."""
    _check_dev(frame, "frame")
    n = frame.numel() if frame_len is None else int(frame_len)
    sd = init_stream_descriptor()
    nb, hl = ctypes.c_uint64(0), ctypes.c_int(0)
    r = lib.lz4mtHipFrameRecords(ctypes.c_void_p(frame.data_ptr()), n, None, 0, ctypes.byref(nb), ctypes.byref(hl),
                                 ctypes.byref(sd), _stream(stream))
    if r != Result.OK:
        raise Lz4MtError(r, "lz4mtHipFrameRecords")
    recs = (ctypes.c_uint64 * (nb.value + 1))()
    r = lib.lz4mtHipFrameRecords(ctypes.c_void_p(frame.data_ptr()), n, recs, nb.value + 1, ctypes.byref(nb),
                                 ctypes.byref(hl), ctypes.byref(sd), _stream(stream))
    if r != Result.OK:
        raise Lz4MtError(r, "lz4mtHipFrameRecords")
    return hl.value, list(recs), sd


def xxh32_chunks(t, chunk=16 << 20, stream=None):
    """XXH32 of each consecutive ``chunk``-byte piece of a device tensor (int32 tensor of digests, same device)."""
    _check_dev(t, "tensor")
    nc = (t.numel() + chunk - 1) // chunk
    d = torch.empty(max(nc, 1), dtype=torch.int32, device=t.device)
    if nc and lib.lz4mtHipXxh32Chunks(ctypes.c_void_p(t.data_ptr()), t.numel(), chunk, ctypes.c_void_p(d.data_ptr()),
                                      _stream(stream)) != 0:
        raise Lz4MtError(Result.ERROR, "lz4mtHipXxh32Chunks")
    return d[:nc]


def decompress_frame(frame, out=None, stream=None, check=True):
    """Decompresses device frame bytes; returns (decoded tensor view, result code)."""
    _check_dev(frame, "frame")
    if out is None:
        out = torch.empty(max(stream_bound(frame, stream), 1), dtype=torch.uint8, device=frame.device)
    sd = init_stream_descriptor()
    osz = ctypes.c_uint64(0)
    r = lib.lz4mtHipDecompressFrame(ctypes.c_void_p(frame.data_ptr()), frame.numel(),
                                    ctypes.c_void_p(out.data_ptr()), out.numel(), ctypes.byref(osz),
                                    ctypes.byref(sd), _stream(stream))
    if check and r != Result.OK:
        raise Lz4MtError(r, "lz4mtHipDecompressFrame")
    return out[:osz.value], r


def gen_synthetic(n, seed=42, device="cuda", stream=None):
    """SURVEY.md App. F synthetic input, generated on the device."""
    t = torch.empty(max(int(n), 1), dtype=torch.uint8, device=device)
    if lib.lz4mtHipGenSynthetic(ctypes.c_void_p(t.data_ptr()), int(n), int(seed), _stream(stream)) != 0:
        raise Lz4MtError(Result.ERROR, "lz4mtHipGenSynthetic")
    return t[:int(n)]


def xxh32(t, stream=None):
    """XXH32 (seed 0) of a device tensor, computed on the device."""
    _check_dev(t, "tensor")
    return int(lib.lz4mtHipXxh32(ctypes.c_void_p(t.data_ptr()), t.numel(), _stream(stream)))


# ---- block-sharded streamed gather (include/lz4mt_hip.h section 4; driven by dist.py)
PACK_HEADER_BYTES = 64


def frame_header(sd):
    """The frame header lz4mtCompress writes for ``sd`` (bytes)."""
    buf = (ctypes.c_uint8 * 20)()
    k = lib.lz4mtHipFrameHeader(ctypes.byref(sd), buf)
    if k < 0:
        raise Lz4MtError(Result.BAD_ARG, "lz4mtHipFrameHeader")
    return bytes(buf[:k])


def shard_workspace(n, sd, device=None):
    """Workspace of an n-byte shard encode (also the root's mirror of such a shard)."""
    nbytes = int(lib.lz4mtHipShardWorkspaceSize(int(n), ctypes.byref(sd)))
    if nbytes == 0:
        raise Lz4MtError(Result.BAD_ARG, "lz4mtHipShardWorkspaceSize (the descriptor does not shard)")
    ws = torch.empty(nbytes, dtype=torch.uint8, device=device or "cuda")
    # the library keeps the Reset -> Encode -> Pack order per workspace
    # address: forget it when the tensor goes, so a later allocation at the
    # same address never inherits "encoded" 
    weakref.finalize(ws, lib.lz4mtHipShardRelease, ctypes.c_void_p(ws.data_ptr()))
    return ws


def shard_pack_bound(n, sd, per_block_cap):
    return int(lib.lz4mtHipShardPackBound(int(n), ctypes.byref(sd), int(per_block_cap)))


def shard_reset(n, sd, ws, stream=None):
    """Zeroes the round state of ``ws`` on ``stream`` (before every encode, and
    stream-ordered before that call's first pack too)."""
    r = lib.lz4mtHipShardReset(int(n), ctypes.byref(sd), ctypes.c_void_p(ws.data_ptr()), ws.numel(), _stream(stream))
    if r != Result.OK:
        raise Lz4MtError(r, "lz4mtHipShardReset")


def shard_encode(src, sd, ws, stream=None):
    """Launches the shard's encode (+ block checksums); asynchronous on
    ``stream``.  ``ws`` must have been reset (``shard_reset``) first."""
    _check_dev(src, "src")
    r = lib.lz4mtHipShardEncode(ctypes.c_void_p(src.data_ptr() if src.numel() else ws.data_ptr()), src.numel(),
                                ctypes.byref(sd), ctypes.c_void_p(ws.data_ptr()), ws.numel(), _stream(stream))
    if r != Result.OK:
        raise Lz4MtError(r, "lz4mtHipShardEncode")


def shard_pack(src, sd, ws, pack, per_block_cap, final, stream=None):
    """One round into ``pack``; asynchronous.  The 64-byte header at pack[:64]
    says how many bytes to send (u64 at 24) and whether the shard is complete
    (u32 at 36, bit 0)."""
    r = lib.lz4mtHipShardPack(ctypes.c_void_p(src.data_ptr() if src.numel() else ws.data_ptr()), src.numel(),
                              ctypes.byref(sd), ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                              ctypes.c_void_p(pack.data_ptr()), pack.numel(), int(per_block_cap), int(bool(final)),
                              _stream(stream))
    if r != Result.OK:
        raise Lz4MtError(r, "lz4mtHipShardPack")


def shard_unpack(pack, n, sd, mirror, stream=None):
    """A received pack (a tensor, or the device address of one) into ``mirror``."""
    ptr = pack if isinstance(pack, int) else pack.data_ptr()
    r = lib.lz4mtHipShardUnpack(ctypes.c_void_p(ptr), int(n), ctypes.byref(sd),
                                ctypes.c_void_p(mirror.data_ptr()), mirror.numel(), _stream(stream))
    if r != Result.OK:
        raise Lz4MtError(r, "lz4mtHipShardUnpack")


def shard_assemble(src, n, sd, ws, body, stream=None):
    """The shard's records into ``body`` (src: the shard's own source, or None for a mirror)."""
    r = lib.lz4mtHipShardAssemble(ctypes.c_void_p(src.data_ptr() if src is not None and src.numel() else None),
                                  int(n), ctypes.byref(sd), ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                                  ctypes.c_void_p(body.data_ptr() if body.numel() else None), body.numel(),
                                  _stream(stream))
    if r != Result.OK:
        raise Lz4MtError(r, "lz4mtHipShardAssemble")


def shard_body_bytes(n, sd, ws, stream=None):
    """Record bytes of a complete shard workspace (synchronises ``stream``)."""
    v = int(lib.lz4mtHipShardBodyBytes(int(n), ctypes.byref(sd), ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                                       _stream(stream)))
    if v == (1 << 64) - 1:
        raise Lz4MtError(Result.ERROR, "lz4mtHipShardBodyBytes")
    return v
