"""Time-boxed random differential campaign (run on the GPU box): random
mixed inputs of random sizes, block sizes, flags, levels and block dependence through the
device frame engine (lz4mtHipCompressFrame / lz4mtHipDecompressFrame), each
frame compared byte for byte with the oracle's frame and each decode with the
input; 40 % of the fast-codec cases (every block size streams since round 6)
also through the callback API in MODE_DEVICE (the streamed compress and
decompress).  Complements the fixed-seed tests with many more shapes.
usage: python tools/fuzz_campaign.py [seconds] [seed]"""
import os
import random
import struct
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import xxhash  # noqa: E402

import lz4mt_amd as L  # noqa: E402
import oracle  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
import make_golden as G  # noqa: E402  (-BD frames from liblz4 1.9.3 with the reference's call sequence)

budget = float(sys.argv[1]) if len(sys.argv) > 1 else 240.0
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rnd = random.Random(seed)
syn = oracle.gen_synthetic(8 << 20, 99)


def piece(out_len):
    k = rnd.randrange(8)
    n = rnd.choice([rnd.randrange(1, 64), rnd.randrange(64, 4096), rnd.randrange(4096, 300_000)])
    if k == 0:
        a = rnd.randrange(len(syn) - n)
        return syn[a:a + n]
    if k == 1:
        return oracle.gen_random(n, rnd.randrange(1 << 30))
    if k == 2:
        return bytes([rnd.randrange(256)]) * n
    if k == 3:   # short period
        p = bytes(rnd.randrange(256) for _ in range(rnd.randrange(1, 9)))
        return (p * (n // len(p) + 1))[:n]
    if k == 4:   # low alphabet
        return bytes(rnd.choice(b"ab") for _ in range(min(n, 20_000)))
    if k == 5 and out_len > 8:   # copy of earlier output, near or beyond 64 KiB
        return None
    if k == 6:
        return oracle.gen_synthetic(min(n, 1 << 20), rnd.randrange(1 << 30))
    return bytes(n)


def gen_input():
    target = rnd.choice([0, 1, 12, 13, rnd.randrange(14, 70_000), rnd.randrange(70_000, 2 << 20),
                         rnd.randrange(2 << 20, 24 << 20), (1 << 20) + rnd.randrange(-2, 3),
                         (4 << 20) * rnd.randrange(1, 5) + rnd.randrange(-1, 2)])
    buf = bytearray()
    while len(buf) < target:
        p = piece(len(buf))
        if p is None:
            d = rnd.choice([rnd.randrange(1, 1000), rnd.randrange(1000, 65536), rnd.randrange(65536, 200_000)])
            d = min(d, len(buf))
            ln = rnd.randrange(4, 5000)
            a = len(buf) - d
            p = bytes(buf[a:a + ln])
        buf += p
    return bytes(buf[:target])


def dev(b):
    t = torch.empty(max(len(b), 1), dtype=torch.uint8, device="cuda")
    if b:
        t[:len(b)].copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
    return t[:len(b)]


def host(t):
    return bytes(t.cpu().numpy().tobytes())


def hc_frame(data, bid, sck, bck, level):
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


t0 = time.time()
cases, nbytes, fails = 0, 0, []
by_level = {}
last = t0
while time.time() - t0 < budget:
    data = gen_input()
    bid = rnd.randrange(4, 8)
    sck, bck = rnd.random() < 0.5, rnd.random() < 0.5
    level = rnd.choice([0, 0, 0, 1, 2, 3, 4, 6, 8, 9, 9, 10, 11, 12])
    bd = rnd.random() < 0.25   # -BD: expected frame from liblz4's stream API
    # 1 / 4 MiB fast -BD blocks: half the cases with LZ4MT_AMD_BD_REFERENCE=1,
    # whose frames are the reference's own (non-decodable) bytes
    refb = bd and level < 3 and bid >= 6 and rnd.random() < 0.5
    if level >= 10 or (bd and level >= 3):
        data = data[:3 << 20]   # the CPU side of the optimal parser / the HC stream is slow
    if bd:   # 1 / 4 MiB fast blocks: the decodable contiguous stream (bugs not copied)
        want = (G.bd_hc_frame_reference(data, bid, sck, bck) if level >= 3
                else G.bd_frame_contiguous(data, bid, sck, bck) if bid >= 6 and not refb
                else G.bd_frame_reference(data, bid, sck, bck))
    else:
        want = (oracle.compress_frame(data, oracle.params(bid, sck, bck)) if level < 3
                else hc_frame(data, bid, sck, bck, level))
    if refb:
        os.environ["LZ4MT_AMD_BD_REFERENCE"] = "1"
    fr = L.compress_frame(dev(data), L.make_sd(bid, sck, bck, block_dependence=bd), level=level)
    os.environ.pop("LZ4MT_AMD_BD_REFERENCE", None)
    got = host(fr)
    ok = got == want
    if ok and refb:   # the reference's bytes: decoding must match the oracle's decode of them
        out, r = L.decompress_frame(fr, out=torch.empty(len(data) + (8 << 20), dtype=torch.uint8, device="cuda"),
                                    check=False)
        rw, ow = oracle.decompress_frame(want, len(data) + (8 << 20))
        ok = (r, host(out)) == (rw, ow)
    elif ok:
        out, r = L.decompress_frame(fr)
        ok = r == 0 and host(out) == data
    if ok and not bd and level < 3 and rnd.random() < 0.4:
        # the callback API in MODE_DEVICE: the streamed compress and decompress
        # (one persistent grid each; lz4mt_frame.cpp compress_streamed /
        # decompress_streamed) against the same oracle frame
        rc, fc = L.compress(data, L.make_sd(bid, sck, bck), mode=L.MODE_DEVICE)
        rd, od, _ = L.decompress(want, len(data) + 64, mode=L.MODE_DEVICE)
        ok = rc == 0 and fc == want and rd == 0 and od == data
        by_level["streamed"] = by_level.get("streamed", 0) + 1
    cases += 1
    nbytes += len(data)
    key = f"{'BDref' if refb else 'BD' if bd else ''}{level}"
    by_level[key] = by_level.get(key, 0) + 1
    if not ok:
        fails.append((cases, len(data), bid, sck, bck, level, bd))
        print(f"MISMATCH case {cases}: n={len(data)} B{bid} sck={sck} bck={bck} level={level} bd={bd}", flush=True)
    if time.time() - last > 30:
        last = time.time()
        print(f"  {cases} cases, {nbytes / 2**20:.0f} MiB, {len(fails)} mismatches", flush=True)
print(f"fuzz campaign seed {seed}: {cases} frames, {nbytes / 2**20:.1f} MiB, levels {dict(sorted(by_level.items()))}, "
      f"{len(fails)} mismatches in {time.time() - t0:.0f} s")
sys.exit(1 if fails else 0)
