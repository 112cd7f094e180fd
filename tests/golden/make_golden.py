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
    json.dump(manifest, open(os.path.join(HERE, "golden.json"), "w"), indent=0)
    print("frames", len(manifest["frames"]), "blocks", len(manifest["blocks"]), "decode", len(manifest["decode"]),
          "crafted", len(manifest["crafted"]), "cli mismatches",
          [(f["input"], f["bid"]) for f in manifest["frames"] if f["cli_body_identical"] is False], "big", big)


if __name__ == "__main__":
    main()
