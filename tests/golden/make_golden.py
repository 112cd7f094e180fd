"""Generates the committed golden fixtures under tests/golden/.

Sources (all present in this image; none is reference code):
  * liblz4.so.1 (lz4 1.9.3, LZ4_versionNumber() == 10903) through ctypes:
    LZ4_compress_limitedOutput / LZ4_decompress_safe — the exact calls
    lz4mt binds (reference src/main.cpp:749-751, 774);
  * python-xxhash 3.x for XXH32 (seed 0);
  * /opt/conda/bin/lz4 (the 1.9.3 CLI) as an independent frame writer for
    cross-checking (-1 -B# [-BX] [--no-frame-crc]).
Frames are assembled here by a small independent writer that follows the
lz4mt frame layout (reference src/lz4mt.cpp:335-457, 898-935).

Run:  python tests/golden/make_golden.py   (rewrites the fixtures)
"""
import ctypes
import hashlib
import json
import os
import random
import struct
import subprocess
import sys
import tempfile

import xxhash

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))
from conftest import bd_data, bd_input  # noqa: E402  (the -BD test input, shared with the GPU tests)
LZ4 = ctypes.CDLL("/lib/x86_64-linux-gnu/liblz4.so.1")
CLI = "/opt/conda/bin/lz4"


def lz4_compress(data, cap):
    dst = ctypes.create_string_buffer(max(cap, 1) + 64)
    n = LZ4.LZ4_compress_limitedOutput(bytes(data), dst, len(data), cap)
    return dst.raw[:n]


def lz4_decompress(block, cap):
    dst = ctypes.create_string_buffer(max(cap, 1) + 64)
    n = LZ4.LZ4_decompress_safe(bytes(block), dst, len(block), cap)
    return n, (dst.raw[:n] if n > 0 else b"")


def xxh(b):
    return xxhash.xxh32(b, seed=0).intdigest()


def frame(data, bid=7, sck=True, bck=False):
    """Independent lz4mt frame writer (layout of reference src/lz4mt.cpp:335-457,898-935)."""
    flg = (1 << 6) | (1 << 5) | (int(bck) << 4) | (int(sck) << 2)
    bd = bid << 4
    desc = bytes([flg, bd])
    out = bytearray(struct.pack("<I", 0x184D2204) + desc + bytes([(xxh(desc) >> 8) & 0xFF]))
    bm = 1 << (8 + 2 * bid)
    for off in range(0, len(data), bm):
        blk = data[off:off + bm]
        c = lz4_compress(blk, len(blk))
        if len(c) == 0:
            out += struct.pack("<I", len(blk) | 0x80000000) + blk
            stored = blk
        else:
            out += struct.pack("<I", len(c)) + c
            stored = c
        if bck:
            out += struct.pack("<I", xxh(stored))
    out += b"\0\0\0\0"
    if sck:
        out += struct.pack("<I", xxh(data))
    return bytes(out)


# ---- block-dependent (-BD) frames ------------------------------------------
def _bd_records(blocks, bck):
    out = bytearray()
    for payload, raw in blocks:
        out += struct.pack("<I", len(payload) | (0x80000000 if raw else 0)) + payload
        if bck:
            out += struct.pack("<I", xxh(payload))
    return bytes(out)


def _bd_header(bid, sck, bck):
    flg = (1 << 6) | (int(bck) << 4) | (int(sck) << 2)   # FLG.5 (block independence) clear
    desc = bytes([flg, bid << 4])
    return struct.pack("<I", 0x184D2204) + desc + bytes([(xxh(desc) >> 8) & 0xFF])


def bd_frame_reference(data, bid, sck, bck):
    """compressBlockDependency (reference src/lz4mt.cpp:460-538) replayed on
    liblz4 1.9.3 with its exact call sequence: a max(bm + 64 KiB, 1088 KiB)
    input buffer, LZ4_resetStreamState, LZ4_compress_limitedOutput_continue
    (cap = inSize - 1), LZ4_slideInputBuffer when the next block would not
    fit.  In 1.9.3 LZ4_slideInputBuffer returns the dictionary pointer, so
    for 1 and 4 MiB blocks the next block is read over its own dictionary
    and the frame does not decode back; 64 and 256 KiB
    blocks round-trip."""
    LZ4.LZ4_slideInputBuffer.restype = ctypes.c_void_p
    bm = 1 << (8 + 2 * bid)
    size = max(bm + 65536, (1024 + 64) * 1024)
    buf = ctypes.create_string_buffer(size)
    base = ctypes.addressof(buf)
    dst = ctypes.create_string_buffer(bm + 64)
    st = ctypes.create_string_buffer(LZ4.LZ4_sizeofStreamState())
    LZ4.LZ4_resetStreamState(st, buf)
    ins, pos, blocks = base, 0, []
    while True:
        if ins + bm > base + size:
            ins = LZ4.LZ4_slideInputBuffer(st)
        chunk = data[pos:pos + bm]
        if not chunk:
            break
        ctypes.memmove(ins, chunk, len(chunk))
        pos += len(chunk)
        n = LZ4.LZ4_compress_limitedOutput_continue(st, ctypes.c_void_p(ins), dst, len(chunk), len(chunk) - 1)
        blocks.append((dst.raw[:n], False) if n > 0 else (chunk, True))
        ins += len(chunk)
    tail = b"\0\0\0\0" + (struct.pack("<I", xxh(data)) if sck else b"")
    return _bd_header(bid, sck, bck) + _bd_records(blocks, bck) + tail


def bd_hc_frame_reference(data, bid, sck, bck):
    """compressBlockDependency at compression level >= 3 (reference
    src/lz4mt.cpp:295-332, 460-538) replayed on liblz4 1.9.3: the legacy HC
    stream -- LZ4_resetStreamStateHC(state, inputBuffer) (which sets the
    stream to lz4hc's default level 9 whatever ctx.compressionLevel says),
    LZ4_compressHC_limitedOutput_continue (cap = inSize - 1), and
    LZ4_slideInputBufferHC when the next block would not fit (in 1.9.3 it
    resets the stream: the next block starts without a dictionary)."""
    LZ4.LZ4_slideInputBufferHC.restype = ctypes.c_void_p
    bm = 1 << (8 + 2 * bid)
    size = max(bm + 65536, (1024 + 64) * 1024)
    buf = ctypes.create_string_buffer(size)
    base = ctypes.addressof(buf)
    dst = ctypes.create_string_buffer(bm + 64)
    st = ctypes.create_string_buffer(LZ4.LZ4_sizeofStreamStateHC())
    assert LZ4.LZ4_resetStreamStateHC(st, buf) == 0
    ins, pos, blocks = base, 0, []
    while True:
        if ins + bm > base + size:
            ins = LZ4.LZ4_slideInputBufferHC(st)
        chunk = data[pos:pos + bm]
        if not chunk:
            break
        ctypes.memmove(ins, chunk, len(chunk))
        pos += len(chunk)
        n = LZ4.LZ4_compressHC_limitedOutput_continue(st, ctypes.c_void_p(ins), dst, len(chunk), len(chunk) - 1)
        blocks.append((dst.raw[:n], False) if n > 0 else (chunk, True))
        ins += len(chunk)
    tail = b"\0\0\0\0" + (struct.pack("<I", xxh(data)) if sck else b"")
    return _bd_header(bid, sck, bck) + _bd_records(blocks, bck) + tail


def bd_frame_contiguous(data, bid, sck, bck):
    """The same stream compressed from one contiguous buffer (every block in
    LZ4 prefix mode after the first), cap = inSize - 1: what the reference's
    loop computes when its dictionary survives (this library's -BD output
    for 1 and 4 MiB blocks)."""
    bm = 1 << (8 + 2 * bid)
    buf = ctypes.create_string_buffer(data, len(data) + 1)
    base = ctypes.addressof(buf)
    dst = ctypes.create_string_buffer(bm + 64)
    st = ctypes.create_string_buffer(LZ4.LZ4_sizeofStreamState())
    LZ4.LZ4_resetStreamState(st, buf)
    blocks = []
    for off in range(0, len(data), bm):
        chunk = data[off:off + bm]
        n = LZ4.LZ4_compress_limitedOutput_continue(st, ctypes.c_void_p(base + off), dst, len(chunk), len(chunk) - 1)
        blocks.append((dst.raw[:n], False) if n > 0 else (chunk, True))
    tail = b"\0\0\0\0" + (struct.pack("<I", xxh(data)) if sck else b"")
    return _bd_header(bid, sck, bck) + _bd_records(blocks, bck) + tail


def bd_decode_reference(frame):
    """decompressBlockDependency (src/lz4mt.cpp:737-845) on liblz4 1.9.3:
    LZ4_decompress_safe_withPrefix64k over a zeroed 64 KiB + block buffer.
    Returns the content or None (a block fails to decode)."""
    bid = (frame[5] >> 4) & 7
    bck = bool(frame[4] & 0x10)
    bm = 1 << (8 + 2 * bid)
    d = ctypes.create_string_buffer(65536 + bm)
    dbase = ctypes.addressof(d)
    dptr, pos, out = dbase + 65536, 7, []
    while True:
        w = struct.unpack_from("<I", frame, pos)[0]
        pos += 4
        if w == 0:
            return b"".join(out)
        n = w & 0x7FFFFFFF
        payload = frame[pos:pos + n]
        pos += n + (4 if bck else 0)
        if w & 0x80000000:
            out.append(payload)
            if n >= 65536:
                ctypes.memmove(dbase, payload[-65536:], 65536)
                dptr = dbase + 65536
                continue
            ctypes.memmove(dptr, payload, n)
            k = n
        else:
            k = LZ4.LZ4_decompress_safe_withPrefix64k(payload, ctypes.c_void_p(dptr), n, bm)
            if k < 0:
                return None
            out.append(ctypes.string_at(dptr, k))
        dptr += k
        if dbase + 65536 + bm - dptr < bm:
            ctypes.memmove(dbase, dptr - 65536, 65536)
            dptr = dbase + 65536


def bd_decompress_reference(frame):
    """lz4mtDecompress on a -BD frame, step for step (src/lz4mt.cpp:938-1011
    frame loop, decompressBlockDependency 737-845) over liblz4 1.9.3's
    LZ4_decompress_safe_withPrefix64k: per block the size word (0 = EOS;
    > blockMax = INVALID_BLOCK_SIZE), the payload, the checksum word and its
    check (BLOCK_CHECKSUM_MISMATCH), then a raw copy or the decode into the
    64 KiB-prefixed buffer (< 0 = DECOMPRESS_FAIL), each block written as it
    is done; after the EOS the content checksum (STREAM_CHECKSUM_MISMATCH).
    Returns (result name, the bytes written)."""
    flg, bid = frame[4], (frame[5] >> 4) & 7
    sck, bck = bool(flg & 0x04), bool(flg & 0x10)
    bm = 1 << (8 + 2 * bid)
    d = ctypes.create_string_buffer(65536 + bm)
    dbase = ctypes.addressof(d)
    dptr, pos, out = dbase + 65536, 7, []

    def u32(at):
        return struct.unpack_from("<I", frame, at)[0] if at + 4 <= len(frame) else None
    while True:
        w = u32(pos)
        if w is None:
            return "CANNOT_READ_BLOCK_SIZE", b"".join(out)
        pos += 4
        if w == 0:
            break
        n = w & 0x7FFFFFFF
        if n > bm:
            return "INVALID_BLOCK_SIZE", b"".join(out)
        if pos + n > len(frame):
            return "CANNOT_READ_BLOCK_DATA", b"".join(out)
        payload = frame[pos:pos + n]
        pos += n
        if bck:
            c = u32(pos)
            if c is None:
                return "CANNOT_READ_BLOCK_CHECKSUM", b"".join(out)
            pos += 4
            if c != xxh(payload):
                return "BLOCK_CHECKSUM_MISMATCH", b"".join(out)
        if w & 0x80000000:
            out.append(payload)
            if n >= 65536:
                ctypes.memmove(dbase, payload[-65536:], 65536)
                dptr = dbase + 65536
                continue
            ctypes.memmove(dptr, payload, n)
            k = n
        else:
            k = LZ4.LZ4_decompress_safe_withPrefix64k(payload, ctypes.c_void_p(dptr), n, bm)
            if k < 0:
                return "DECOMPRESS_FAIL", b"".join(out)
            out.append(ctypes.string_at(dptr, k))
        dptr += k
        if dbase + 65536 + bm - dptr < bm:
            ctypes.memmove(dbase, dptr - 65536, 65536)
            dptr = dbase + 65536
    content = b"".join(out)
    if sck:
        c = u32(pos)
        if c is None:
            return "CANNOT_READ_STREAM_CHECKSUM", content
        if c != xxh(content):
            return "STREAM_CHECKSUM_MISMATCH", content
    return "OK", content


# Frames the reference itself writes with 1 and 4 MiB blocks (bd_frame_reference:
# every block after the first is read over its own dictionary, see
# DESIGN.md), and what lz4mtDecompress does with them: users with such -BD
# archives feed exactly these bytes in.  (name, bytes, seed, id, sck, bck)
BD_REF_DECODE = [  # (name, bytes, seed, id, sck, bck, input: "bd" = bd_input, "appf" = App. F)
    ("bdref_b6_SX", (2 << 20) + 100_000, 71, 6, True, True, "bd"),          # decodes back, other bytes than ours
    ("bdref_b6_appf_SX", (2 << 20) + 100_000, 42, 6, True, True, "appf"),   # STREAM_CHECKSUM_MISMATCH
    ("bdref_b6_appf_sX", (2 << 20) + 100_000, 42, 6, False, True, "appf"),  # OK, but not the input
    ("bdref_b7_Sx", (4 << 20) + 200_000, 73, 7, True, False, "bd"),
    ("bdref_b7_sx", (4 << 20) + 150_000, 74, 7, False, False, "bd"),
]


def bd_ref_decode_main(manifest):
    from oracle import gen_synthetic
    manifest["bd_ref_decode"] = []
    for name, n, seed, bid, sck, bck, kind in BD_REF_DECODE:
        data = bd_input(n, seed) if kind == "bd" else gen_synthetic(n, seed)
        f = bd_frame_reference(data, bid, sck, bck)
        res, out = bd_decompress_reference(f)
        open(os.path.join(HERE, "frames", f"{name}.lz4"), "wb").write(f)
        manifest["bd_ref_decode"].append({
            "name": name, "bytes": n, "seed": seed, "kind": kind, "bid": bid, "stream_checksum": sck,
            "block_checksum": bck, "file": f"frames/{name}.lz4", "size": len(f), "xxh32": xxh(f),
            "content_xxh32": xxh(data), "result": res, "out_bytes": len(out), "out_xxh32": xxh(out),
            "roundtrips": out == data, "contiguous_identical": f == bd_frame_contiguous(data, bid, sck, bck)})


# Known answers (size + XXH32) of frames the reference writes with 1 and 4 MiB
# blocks over several FULL blocks (each read over its own dictionary from
# the second on), for the opt-in LZ4MT_AMD_BD_REFERENCE=1 compressor:
# (name, bytes, seed, id, sck, bck, input: "bd" = bd_input, "appf" = App. F)
BD_REF_KNOWN = [
    ("bdrefk_b6_9m", 9_437_184 + 4321, 23, 6, False, True, "bd"),
    ("bdrefk_b6_4m_exact", 4 << 20, 5, 6, True, True, "appf"),   # no short last block
    ("bdrefk_b7_9m", 9_437_184 + 4321, 24, 7, True, False, "bd"),
    ("bdrefk_b7_appf_17m", (17 << 20) + 99, 42, 7, False, True, "appf"),
]


def bd_ref_known_main(manifest):
    from oracle import gen_synthetic
    manifest["bd_ref_known"] = []
    for name, n, seed, bid, sck, bck, kind in BD_REF_KNOWN:
        data = bd_input(n, seed) if kind == "bd" else gen_synthetic(n, seed)
        f = bd_frame_reference(data, bid, sck, bck)
        manifest["bd_ref_known"].append({
            "name": name, "bytes": n, "seed": seed, "kind": kind, "bid": bid, "stream_checksum": sck,
            "block_checksum": bck, "size": len(f), "xxh32": xxh(f), "content_xxh32": xxh(data),
            "contiguous_identical": f == bd_frame_contiguous(data, bid, sck, bck)})


BD_CASES = [  # (name, bytes, seed, block id, stream checksum, block checksum[, input kind])
    ("bd_b4_sX", 1_500_000, 11, 4, False, True), ("bd_b4_SX", 1_500_000, 11, 4, True, True),
    ("bd_b5_Sx", 1_500_000, 12, 5, True, False),
    # edges: empty, shorter than a match, exactly one block and one byte more,
    # a short last block, all-zero, incompressible (every block raw), mixed
    ("bd_e0", 0, 31, 4, True, True), ("bd_e1", 1, 32, 4, False, True), ("bd_e13", 13, 33, 5, True, False),
    ("bd_e64k", 65536, 34, 4, False, True), ("bd_e64k1", 65537, 35, 4, True, True),
    ("bd_e3b", 3 * 65536 + 5, 36, 4, False, False), ("bd_zero", 400_000, 37, 4, False, True, "zeros"),
    ("bd_rand", 300_000, 38, 4, True, True, "random"), ("bd_mix4", 1_300_000, 39, 4, False, True, "mixed"),
    ("bd_mix5", 1_300_000, 40, 5, True, True, "mixed"),
]
BD_HC_CASES = [  # -BD at level >= 3 (lz4hc level 9 stream): (name, bytes, seed, id, sck, bck[, kind])
    ("bdhc_b4_sX", 1_500_000, 51, 4, False, True), ("bdhc_b5_Sx", 1_500_000, 52, 5, True, False),
    ("bdhc_b6_SX", 2_500_000, 53, 6, True, True), ("bdhc_e13", 13, 54, 4, False, True),
    ("bdhc_e64k1", 65537, 55, 4, True, True), ("bdhc_mix4", 1_300_000, 56, 4, False, True, "mixed"),
    ("bdhc_zero", 300_000, 57, 5, False, True, "zeros"), ("bdhc_rand", 200_000, 58, 4, True, True, "random"),
]
BD_HC_KNOWN = [  # (name, bytes, seed, id, sck, bck): size + XXH32 only
    ("bdhc_b7_9m", 9_437_184 + 4321, 61, 7, True, True), ("bdhc_b4_9m", 9_437_184 + 4321, 62, 4, False, True),
]
BD_KNOWN = [  # larger -BD frames pinned by size + XXH32 only: (name, bytes, seed, id, sck, bck, writer)
    ("bd_b4_9m", 9_437_184 + 4321, 21, 4, False, True, "reference"),
    ("bd_b5_9m", 9_437_184 + 4321, 22, 5, True, True, "reference"),
    ("bd_b6_9m", 9_437_184 + 4321, 23, 6, False, True, "contiguous"),
    ("bd_b7_9m", 9_437_184 + 4321, 24, 7, True, False, "contiguous"),
]


def bd_hc_main(manifest):
    manifest["bd_hc_frames"], manifest["bd_hc_known"] = [], []
    for name, n, seed, bid, sck, bck, *kind in BD_HC_CASES:
        entry = {"name": name, "bytes": n, "seed": seed, "bid": bid, "stream_checksum": sck, "block_checksum": bck}
        if kind:
            entry["kind"] = kind[0]
        data = bd_data(entry)
        f = bd_hc_frame_reference(data, bid, sck, bck)
        assert bd_decode_reference(f) == data, name
        open(os.path.join(HERE, "frames", f"{name}.lz4"), "wb").write(f)
        entry.update({"file": f"frames/{name}.lz4", "size": len(f), "xxh32": xxh(f), "content_xxh32": xxh(data)})
        manifest["bd_hc_frames"].append(entry)
    for name, n, seed, bid, sck, bck in BD_HC_KNOWN:
        data = bd_input(n, seed)
        f = bd_hc_frame_reference(data, bid, sck, bck)
        assert bd_decode_reference(f) == data, name
        manifest["bd_hc_known"].append({"name": name, "bytes": n, "seed": seed, "bid": bid, "stream_checksum": sck,
                                        "block_checksum": bck, "size": len(f), "xxh32": xxh(f),
                                        "content_xxh32": xxh(data)})


def bd_main(manifest):
    manifest["bd_frames"], manifest["bd_known"] = [], []
    for name, n, seed, bid, sck, bck, *kind in BD_CASES:
        entry = {"name": name, "bytes": n, "seed": seed, "bid": bid, "stream_checksum": sck, "block_checksum": bck}
        if kind:
            entry["kind"] = kind[0]
        data = bd_data(entry)
        f = bd_frame_reference(data, bid, sck, bck)
        assert bd_decode_reference(f) == data, name
        open(os.path.join(HERE, "frames", f"{name}.lz4"), "wb").write(f)
        entry.update({"file": f"frames/{name}.lz4", "size": len(f), "xxh32": xxh(f), "content_xxh32": xxh(data)})
        manifest["bd_frames"].append(entry)
    for name, n, seed, bid, sck, bck, writer in BD_KNOWN:
        data = bd_input(n, seed)
        f = (bd_frame_reference if writer == "reference" else bd_frame_contiguous)(data, bid, sck, bck)
        ok = bd_decode_reference(f) == data
        assert ok, name
        ref = bd_frame_reference(data, bid, sck, bck)
        manifest["bd_known"].append({"name": name, "bytes": n, "seed": seed, "bid": bid, "stream_checksum": sck,
                                     "block_checksum": bck, "writer": writer, "size": len(f), "xxh32": xxh(f),
                                     "content_xxh32": xxh(data), "reference_frame_identical": ref == f,
                                     "reference_frame_roundtrips": bd_decode_reference(ref) == data})


def cli_frame(data, bid, sck, bck):
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "in"), os.path.join(d, "out.lz4")
        open(src, "wb").write(data)
        args = [CLI, "-1", f"-B{bid}", "-q", "-q", "-f"] + (["-BX"] if bck else []) + ([] if sck else ["--no-frame-crc"])
        if subprocess.run(args + [src, dst]).returncode != 0:
            return None   # the 1.9.3 CLI refuses some -B4 inputs (ERROR_dstMaxSize_tooSmall)
        return open(dst, "rb").read()


def inputs():
    from oracle import gen_random, gen_synthetic  # pinned generator (App. F verified)
    rnd = random.Random(1234)
    syn = gen_synthetic(400_000, 42)
    text = (b"lz4mt is a multithreaded LZ4 frame compressor; " * 400)
    cases = {
        "empty": b"",
        "one": b"x",
        "eleven": b"hello world",
        "twelve": b"abcabcabcabc",
        "thirteen": b"abcabcabcabca",
        "text1k": text[:1000],
        "text20k": text,
        "zeros300k": bytes(300_000),
        "random100k": gen_random(100_000, 7),
        "syn65535": syn[:65535],
        "syn65546": syn[:65546],
        "syn65547": syn[:65547],
        "syn65548": syn[:65548],
        "syn300k": syn[:300_000],
        "ab5000": bytes(rnd.choice(b"ab") for _ in range(5000)),
        "runs": b"".join(bytes([rnd.randrange(256)]) * rnd.randrange(1, 300) for _ in range(400)),
    }
    return cases


FLAG_SETS = [  # (block id, stream checksum, block checksum)
    (7, True, False), (7, False, True), (7, True, True), (4, True, False), (4, False, True), (5, True, False),
    (6, False, True),
]


def main():
    cases = inputs()
    os.makedirs(os.path.join(HERE, "frames"), exist_ok=True)
    manifest = {"lz4_version": LZ4.LZ4_versionNumber(), "inputs": {}, "frames": [], "blocks": [], "decode": []}
    for name, data in cases.items():
        path = os.path.join(HERE, "frames", f"{name}.bin")
        open(path, "wb").write(data)
        manifest["inputs"][name] = {"file": f"frames/{name}.bin", "size": len(data), "xxh32": xxh(data)}
        for bid, sck, bck in FLAG_SETS:
            f = frame(data, bid, sck, bck)
            fname = f"frames/{name}.B{bid}{'S' if sck else 's'}{'X' if bck else 'x'}.lz4"
            open(os.path.join(HERE, fname), "wb").write(f)
            cli = cli_frame(data, bid, sck, bck)
            manifest["frames"].append({"input": name, "bid": bid, "stream_checksum": sck, "block_checksum": bck,
                                       "file": fname, "size": len(f), "xxh32": xxh(f),
                                       "cli_identical": None if cli is None else cli == f,
                                       # the CLI shrinks BD for inputs smaller than the block: compare bodies
                                       "cli_body_identical": None if cli is None else cli[7:] == f[7:]})
        # block-level vectors: cap = n (lz4mt), n-1 (LZ4F), bound (notLimited)
        for cap in sorted({len(data), max(len(data) - 1, 0), len(data) + len(data) // 255 + 16}):
            blk = data[:70_000]
            c = lz4_compress(blk, min(cap, len(blk) + len(blk) // 255 + 16))
            manifest["blocks"].append({"input": name, "n": len(blk), "cap": min(cap, len(blk) + len(blk) // 255 + 16),
                                       "ret": len(c), "sha1": hashlib.sha1(c).hexdigest()})
    # decoder acceptance vectors: valid blocks under many capacities + mutations
    rnd = random.Random(99)
    srcs = [cases["text1k"], cases["syn300k"][:20000], cases["zeros300k"], cases["runs"], cases["ab5000"],
            cases["thirteen"]]
    blob = bytearray()
    for si, data in enumerate(srcs):
        blk = lz4_compress(data, len(data) + len(data) // 255 + 16)
        caps = [len(data), len(data) + 1, len(data) + 5, len(data) + 12, len(data) + 32, len(data) + 64,
                len(data) + 100, 1 << 16, 4 << 20]
        variants = [("valid", blk)]
        for t in range(60):
            m = bytearray(blk)
            k = rnd.randrange(4)
            if not m:
                break
            if k == 0:
                m[rnd.randrange(len(m))] = rnd.randrange(256)
            elif k == 1:
                m = m[:rnd.randrange(len(m))]
            elif k == 2:
                m += bytes(rnd.randrange(256) for _ in range(rnd.randrange(1, 20)))
            else:
                for _ in range(5):
                    m[rnd.randrange(len(m))] = rnd.randrange(256)
            variants.append((f"mut{t}", bytes(m)))
        for vname, v in variants:
            off = len(blob)
            blob += v
            for cap in caps:
                r, out = lz4_decompress(v, cap)
                manifest["decode"].append({"src": si, "variant": vname, "off": off, "len": len(v), "cap": cap,
                                           "ret": r, "out_xxh32": xxh(out) if r >= 0 else None})
    open(os.path.join(HERE, "decode_blocks.bin"), "wb").write(bytes(blob))
    big = len(blob)
    # crafted acceptance edge cases
    crafted = {
        "empty": b"",
        "zero_token": b"\x00",
        "lit8_m4_lit5": bytes([0x80]) + b"ABCDEFGH" + b"\x08\x00" + bytes([0x50]) + b"12345",
        "lit8_m18_lit5": bytes([0x8F]) + b"ABCDEFGH" + b"\x08\x00" + b"\x03" + bytes([0x50]) + b"12345",
        "offset0": bytes([0x84]) + b"ABCDEFGH" + b"\x00\x00" + bytes([0x50]) + b"12345",
        "offset_before_start": bytes([0x40]) + b"ABCD" + b"\x09\x00" + bytes([0x50]) + b"12345",
        "ends_in_match": bytes([0x80]) + b"ABCDEFGH" + b"\x08\x00",
        "short_last_lits": bytes([0x80]) + b"ABCDEFGH" + b"\x08\x00" + bytes([0x30]) + b"123",
        "trailing_garbage": bytes([0x50]) + b"12345" + b"zz",
        "rle_long": bytes([0x1F]) + b"a" + b"\x01\x00" + b"\xff" * 20 + b"\x10" + bytes([0x50]) + b"12345",
    }
    manifest["crafted"] = []
    for name, blk in crafted.items():
        for cap in (0, 1, 16, 17, 19, 20, 30, 31, 64, 100, 8192, 4 << 20):
            r, out = lz4_decompress(blk, cap)
            manifest["crafted"].append({"name": name, "block_hex": blk.hex(), "cap": cap, "ret": r,
                                        "out_hex": out.hex() if r > 0 and len(out) <= 64 else None,
                                        "out_xxh32": xxh(out) if r >= 0 else None})
    # LZ4-HC block vectors: LZ4_compressHC2_limitedOutput = LZ4_compress_HC
    # (the reference's codec for levels >= 3, src/main.cpp:778-785)
    LZ4.LZ4_compress_HC.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    manifest["hc_blocks"] = []
    hc_inputs = dict(cases)
    hc_inputs["bdmix300k"] = bd_input(300_000, 31)
    for name, data in hc_inputs.items():
        blk = data[:300_000]
        for level in (3, 4, 6, 8, 9, 10, 11, 12):   # 10..12: the optimal parser (the CLI's -A asks for 17 = 12)
            for cap in sorted({len(blk), max(len(blk) - 1, 0)}):
                dst = ctypes.create_string_buffer(max(cap, 1) + len(blk) // 255 + 64)
                r = LZ4.LZ4_compress_HC(blk, dst, len(blk), cap, level)
                manifest["hc_blocks"].append({"input": name, "n": len(blk), "cap": cap, "level": level, "ret": r,
                                              "sha1": hashlib.sha1(dst.raw[:r]).hexdigest()})
    bd_main(manifest)
    bd_hc_main(manifest)
    bd_ref_decode_main(manifest)
    json.dump(manifest, open(os.path.join(HERE, "golden.json"), "w"), indent=0)
    print("frames", len(manifest["frames"]), "blocks", len(manifest["blocks"]), "decode", len(manifest["decode"]),
          "crafted", len(manifest["crafted"]), "cli mismatches",
          [(f["input"], f["bid"]) for f in manifest["frames"] if f["cli_body_identical"] is False], "big", big)


if __name__ == "__main__":
    if "--bd-ref-known" in sys.argv:   # add / refresh only that section of golden.json
        path = os.path.join(HERE, "golden.json")
        m = json.load(open(path))
        bd_ref_known_main(m)
        json.dump(m, open(path, "w"), indent=0)
        print(json.dumps(m["bd_ref_known"], indent=1))
    elif "--bd-ref-decode" in sys.argv:   # add / refresh only that section of golden.json
        path = os.path.join(HERE, "golden.json")
        m = json.load(open(path))
        bd_ref_decode_main(m)
        json.dump(m, open(path, "w"), indent=0)
        print(json.dumps(m["bd_ref_decode"], indent=1))
    else:
        main()
