"""ctypes wrapper of oracle/liblz4mt_oracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker / CPU baseline.  The product
(lz4mt_amd/) never imports it.  See lz4_oracle.h for what it restates and
how it is pinned (liblz4 1.9.3, python-xxhash, lz4 CLI).
"""
import ctypes
import struct
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liblz4mt_oracle.so")


class FrameParams(ctypes.Structure):
    _fields_ = [("streamChecksum", ctypes.c_int), ("blockChecksum", ctypes.c_int), ("blockMaxId", ctypes.c_int),
                ("streamSizeFlag", ctypes.c_int), ("streamSize", ctypes.c_uint64)]


class KnownAnswer(ctypes.Structure):
    _fields_ = [("frameSize", ctypes.c_uint64), ("frameXxh32", ctypes.c_uint32), ("frameChunks", ctypes.c_uint32),
                ("contentXxh32", ctypes.c_uint32), ("contentChunks", ctypes.c_uint32)]


def build():
    subprocess.run(["make", "-C", HERE, "-s"], check=True)


def _load():
    if not os.path.exists(LIB_PATH):
        build()
    lib = ctypes.CDLL(LIB_PATH)
    u8p, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.orc_xxh32.restype = ctypes.c_uint32
    lib.orc_xxh32.argtypes = [u8p, sz, ctypes.c_uint32]
    lib.orc_lz4_compress_bound.restype = ctypes.c_int
    lib.orc_lz4_compress.argtypes = [u8p, u8p, ctypes.c_int, ctypes.c_int]
    lib.orc_lz4_decompress_safe.argtypes = [u8p, u8p, ctypes.c_int, ctypes.c_int]
    lib.orc_lz4hc_compress.argtypes = [u8p, u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.orc_lz4_decompress_safe_prefix64k.argtypes = [u8p, u8p, ctypes.c_int, ctypes.c_int]
    lib.orc_frame_bound.restype = sz
    lib.orc_frame_bound.argtypes = [sz, ctypes.POINTER(FrameParams)]
    lib.orc_frame_compress.restype = sz
    lib.orc_frame_compress.argtypes = [u8p, sz, u8p, ctypes.POINTER(FrameParams), ctypes.c_int]
    lib.orc_frame_decompress.argtypes = [u8p, sz, u8p, sz, ctypes.POINTER(sz), ctypes.c_int]
    lib.orc_gen_synthetic.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64]
    lib.orc_gen_random.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64]
    lib.orc_pipeline_roundtrip.argtypes = [u8p, sz, ctypes.POINTER(FrameParams), ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_double), ctypes.POINTER(sz)]
    lib.orc_pipeline_roundtrip_codec.argtypes = [u8p, sz, ctypes.POINTER(FrameParams), ctypes.c_int,
                                                 ctypes.POINTER(ctypes.c_double), ctypes.POINTER(sz), u8p, u8p]
    lib.orc_bd_hc_body.restype = ctypes.c_int64
    lib.orc_bd_hc_body.argtypes = [u8p, sz, ctypes.c_int, ctypes.c_int, u8p]
    lib.orc_hc_codec_set.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.orc_bd_roundtrip.argtypes = [u8p, sz, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_double), ctypes.POINTER(sz)]
    lib.orc_stream_known_answer.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(FrameParams),
                                            ctypes.c_int, ctypes.c_uint64, ctypes.POINTER(KnownAnswer)]
    return lib


lib = _load()


def _buf(data):
    return ctypes.create_string_buffer(bytes(data), max(len(data), 1))


def xxh32(data, seed=0):
    return lib.orc_xxh32(_buf(data), len(data), seed)


def compress_block(data, cap=None):
    """LZ4_compress_limitedOutput(src, dst, n, cap) restated; b'' when it does not fit."""
    cap = len(data) if cap is None else cap
    dst = ctypes.create_string_buffer(max(cap, lib.orc_lz4_compress_bound(len(data))) + 16)
    n = lib.orc_lz4_compress(_buf(data), dst, len(data), cap)
    return dst.raw[:n]


def compress_block_hc(data, cap=None, level=9):
    """LZ4_compressHC2_limitedOutput(src, dst, n, cap, level) restated (levels 1..9 hashChain,
    10..12 and above the optimal parser); b'' when it does not fit."""
    cap = len(data) if cap is None else cap
    dst = ctypes.create_string_buffer(max(cap, lib.orc_lz4_compress_bound(len(data))) + 16)
    n = lib.orc_lz4hc_compress(_buf(data), dst, len(data), cap, level)
    return dst.raw[:n]


def bd_hc_frame(data, block_max_id, stream_checksum, block_checksum):
    """A -BD frame at compression level >= 3 (compressBlockDependency over
    the legacy HC stream, reference src/lz4mt.cpp:295-332, 460-538):
    header (FLG.5 = 0), orc_bd_hc_body's records, end mark, [content XXH32]."""
    flg = 0x40 | (0x10 if block_checksum else 0) | (0x04 if stream_checksum else 0)
    desc = bytes([flg, block_max_id << 4])
    hdr = struct.pack("<I", 0x184D2204) + desc + bytes([(xxh32(desc) >> 8) & 0xFF])
    nb = (len(data) + (1 << (8 + 2 * block_max_id)) - 1) >> (8 + 2 * block_max_id)
    dst = ctypes.create_string_buffer(len(data) + 8 * nb + 16)
    n = lib.orc_bd_hc_body(_buf(data), len(data), block_max_id, int(block_checksum), dst)
    tail = b"\0\0\0\0" + (struct.pack("<I", xxh32(data)) if stream_checksum else b"")
    return hdr + dst.raw[:n] + tail


def decompress_block(block, cap):
    """LZ4_decompress_safe restated: (ret, bytes)."""
    dst = ctypes.create_string_buffer(max(cap, 1) + 16)
    n = lib.orc_lz4_decompress_safe(_buf(block), dst, len(block), cap)
    return n, (dst.raw[:n] if n > 0 else b"")


def decompress_block_prefix64k(block, cap, prefix=b""):
    """LZ4_decompress_safe_withPrefix64k restated: (ret, bytes); ``prefix`` =
    the history before the block (zero-padded to 64 KiB on the left)."""
    hist = (bytes(65536) + bytes(prefix))[-65536:]
    buf = ctypes.create_string_buffer(hist + bytes(max(cap, 1) + 16), 65536 + max(cap, 1) + 16)
    n = lib.orc_lz4_decompress_safe_prefix64k(_buf(block), ctypes.byref(buf, 65536), len(block), cap)
    return n, (buf.raw[65536:65536 + n] if n > 0 else b"")


def params(block_max_id=7, stream_checksum=True, block_checksum=False, stream_size=None):
    return FrameParams(1 if stream_checksum else 0, 1 if block_checksum else 0, block_max_id,
                       0 if stream_size is None else 1, stream_size or 0)


def compress_frame(data, p=None, threads=8):
    p = p or params()
    cap = lib.orc_frame_bound(len(data), ctypes.byref(p))
    dst = ctypes.create_string_buffer(cap)
    n = lib.orc_frame_compress(_buf(data), len(data), dst, ctypes.byref(p), threads)
    return dst.raw[:n]


def decompress_frame(frame, out_cap, threads=8):
    """(result code, decoded bytes) with lz4mtDecompress semantics."""
    dst = ctypes.create_string_buffer(max(out_cap, 1))
    osz = ctypes.c_size_t(0)
    r = lib.orc_frame_decompress(_buf(frame), len(frame), dst, out_cap, ctypes.byref(osz), threads)
    return r, dst.raw[:osz.value]


def gen_synthetic(n, seed=42):
    b = ctypes.create_string_buffer(max(n, 1))
    lib.orc_gen_synthetic(b, n, seed)
    return b.raw[:n]


def gen_random(n, seed=7):
    b = ctypes.create_string_buffer(max(n, 1))
    lib.orc_gen_random(b, n, seed)
    return b.raw[:n]


def pipeline_roundtrip(data_buf, n, p, threads, codec=None):
    """lz4mt-shaped CPU pipeline timing: (compress_s, decompress_s, frame_bytes).

    ``codec`` = (compress_fn_ptr, decompress_fn_ptr) with the LZ4 signatures
    lz4mt binds (e.g. from liblz4.so.1, see ``liblz4_codec``); None = this
    restatement."""
    secs = (ctypes.c_double * 2)()
    fs = ctypes.c_size_t(0)
    cf, df = codec if codec else (None, None)
    err = lib.orc_pipeline_roundtrip_codec(data_buf, n, ctypes.byref(p), threads, secs, ctypes.byref(fs), cf, df)
    if err:
        raise RuntimeError("oracle pipeline decode error")
    return secs[0], secs[1], fs.value


def liblz4_codec(path="liblz4.so.1"):
    """(compress, decompress, version) function pointers of the system liblz4
    -- the library lz4mt links (src/main.cpp:749-751, 774) -- or None."""
    try:
        lz = ctypes.CDLL(path)
    except OSError:
        return None
    lz.LZ4_versionNumber.restype = ctypes.c_int
    v = lz.LZ4_versionNumber()
    cf = ctypes.cast(lz.LZ4_compress_limitedOutput, ctypes.c_void_p).value
    df = ctypes.cast(lz.LZ4_decompress_safe, ctypes.c_void_p).value
    return (cf, df), f"{v // 10000}.{v // 100 % 100}.{v % 100}", lz


def hc_codec(level, lz=None):
    """(compress, decompress) pointers for the pipeline with lz4mt's level >= 3
    codec, LZ4_compressHC2_limitedOutput(src, dst, n, cap, level)
    (src/main.cpp:778-785), from liblz4 ``lz`` (a ctypes CDLL) or, when None,
    this restatement (orc_lz4hc_compress); decompression is the fast
    codec's (the same LZ4 block format)."""
    fn = None
    if lz is not None:
        fn = ctypes.cast(getattr(lz, "LZ4_compressHC2_limitedOutput", None) or lz.LZ4_compress_HC,
                         ctypes.c_void_p).value
    lib.orc_hc_codec_set(fn, level)
    tramp = ctypes.cast(lib.orc_hc_compress_tramp, ctypes.c_void_p).value
    dec = ctypes.cast(lz.LZ4_decompress_safe, ctypes.c_void_p).value if lz is not None else None
    return tramp, dec


def bd_roundtrip(data_buf, n, block_max_id, stream_checksum, block_checksum, lz, hc=False):
    """Single-thread -BD round trip over liblz4's stream API (the reference's
    compressBlockDependency / decompressBlockDependency shape; ``hc``: its
    level >= 3 HC stream): (compress_s, decompress_s, frame_bytes)."""
    names = (("LZ4_createStreamHC", "LZ4_freeStreamHC", "LZ4_compress_HC_continue") if hc else
             ("LZ4_createStream", "LZ4_freeStream", "LZ4_compress_fast_continue")) + ("LZ4_decompress_safe_usingDict",)
    ptr = [ctypes.cast(getattr(lz, f), ctypes.c_void_p).value for f in names]
    secs = (ctypes.c_double * 2)()
    fs = ctypes.c_size_t(0)
    if lib.orc_bd_roundtrip(data_buf, n, block_max_id, int(stream_checksum), int(block_checksum), *ptr, int(hc),
                            secs, ctypes.byref(fs)) != 0:
        raise RuntimeError("-BD CPU round trip failed")
    return secs[0], secs[1], fs.value


def known_answer(n, p, seed=42, chunk=16 << 20, threads=8):
    """Streamed known answer of the App. F input (``orc_stream_known_answer``)."""
    ka = KnownAnswer()
    if lib.orc_stream_known_answer(n, seed, ctypes.byref(p), threads, chunk, ctypes.byref(ka)) != 0:
        raise RuntimeError("known answer failed")
    return {"frame_size": ka.frameSize, "frame_xxh32": ka.frameXxh32, "frame_chunks": ka.frameChunks,
            "content_xxh32": ka.contentXxh32, "content_chunks": ka.contentChunks}
