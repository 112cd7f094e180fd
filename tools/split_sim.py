"""Overlap a split parse of 4 MiB blocks would need (tools/split_sim.c):
for stream starts s inside App. F blocks, the distance from s to the first
loop top from which the cold parse started at s and the block's real parse
agree (same hit probe and match end per sequence) for 64 KiB -- the bytes
stream j-1 must parse past its end before stream j's output can be trusted.
usage: python tools/split_sim.py [blocks=8] [streams=8]"""
import ctypes
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402  (the App. F generator; test infrastructure)

so = "/tmp/split_sim.so"
subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-o", so,
                       os.path.join(os.path.dirname(os.path.abspath(__file__)), "split_sim.c")])
lib = ctypes.CDLL(so)
BM = 4 << 20
blocks = int(sys.argv[1]) if len(sys.argv) > 1 else 8
streams = int(sys.argv[2]) if len(sys.argv) > 2 else 8
data = oracle.gen_synthetic(BM * blocks, 42)
CAP = 1 << 20
H = (ctypes.c_uint32 * CAP)
res = []
for b in range(blocks):
    blk = data[b * BM:(b + 1) * BM]
    buf = ctypes.create_string_buffer(blk, BM)
    eh, ee = H(), H()
    ne = lib.parse(buf, BM, 0, eh, ee, CAP, None)
    E = {ee[i]: i for i in range(ne)}
    if b == 0:   # the real parse is lz4's: its encoded size equals the oracle's (App. A restatement)
        st = H()
        lib.parse(buf, BM, 0, eh, ee, CAP, st)
        size, anc = 0, 0
        for i in range(ne):
            lit, ml = st[i] - anc, ee[i] - st[i] - 4
            size += 1 + (lit + 240) // 255 * (lit >= 15) + lit + 2 + (ml + 240) // 255 * (ml >= 15)
            anc = ee[i]
        run = BM - anc
        size += 1 + (run + 240) // 255 * (run >= 15) + run
        want = len(oracle.compress_block(blk, BM))
        print(f"block 0: {ne} sequences, encoded {size} B, oracle {want} B", flush=True)
        assert size == want
    for j in range(1, streams):
        s = j * BM // streams
        ch, ce = H(), H()
        nc = lib.parse(buf, BM, s, ch, ce, CAP, None)
        meet = conv = None
        i = 0
        while i < nc:   # candidate meeting points: loop tops of the cold parse the real one also passes
            m = ce[i]
            if m in E:
                e = E[m]
                a, c, ok = e + 1, i + 1, True
                while c < nc and a < ne and ce[c] <= m + 65536:
                    if (ch[c], ce[c]) != (eh[a], ee[a]):
                        ok = False
                        break
                    a, c = a + 1, c + 1
                if ok:
                    meet, conv = m, (ce[c] if c < nc else BM)
                    break
                meet = meet or m
            i += 1
        res.append((b, j, s, None if conv is None else conv - s, None if meet is None else meet - s))
        print(f"block {b} stream {j} at {s >> 10} KiB: first common loop top +{(meet - s) if meet else -1} B, "
              f"agreement from then for 64 KiB ends +{(conv - s) if conv else -1} B", flush=True)
ov = [r[3] for r in res if r[3] is not None]
print(f"overlap needed: mean {sum(ov) / len(ov) / 1024:.1f} KiB, max {max(ov) / 1024:.1f} KiB over {len(ov)} "
      f"boundaries ({len(res) - len(ov)} never converged)")
