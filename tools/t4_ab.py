"""B4 A/B: k_encode16 (byU16 split table, 8-bit tags,
LDS source ring, dummy slots: 26.3 KiB, 6 waves per CU) against k_encode16t4
(4-bit tags, no ring, no dummies: 20 KiB, 8 waves per CU; LZ4MT_AMD_ENC=t4).
Parity first (frames of App. F and collision-heavy mixed input against the
CPU oracle, and the 8 GiB frame of both kernels compared), then encode
kernel times at 8 GiB B4, alternating, three passes each.
usage: python tools/t4_ab.py"""
import ctypes
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402
import oracle  # noqa: E402


def setv(v):
    if v == "t4":
        os.environ["LZ4MT_AMD_ENC"] = "t4"
    else:
        os.environ.pop("LZ4MT_AMD_ENC", None)


rnd = random.Random(5)
syn = oracle.gen_synthetic(12 << 20, 9)
mixed = bytearray(syn[:6 << 20])
for s in range(0, len(mixed), 1 << 20):
    for i in range(s, s + 200_000):
        mixed[i] = 97 + rnd.randrange(3)
bad = []
for v in ("base", "t4"):
    setv(v)
    for label, data in (("appf", syn), ("mixed", bytes(mixed)), ("random", oracle.gen_random(3 << 20, 4))):
        src = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        for sck, bck in ((False, True), (True, False)):
            got = bytes(L.compress_frame(src, L.make_sd(4, sck, bck)).cpu().numpy().tobytes())
            if got != oracle.compress_frame(data, oracle.params(4, sck, bck)):
                bad.append((v, label, sck, bck))
print("parity vs oracle:", "OK" if not bad else bad, flush=True)
n = 8 << 30
src = L.gen_synthetic(n)
sd = L.make_sd(4, False, True)
dig = {}
for v in ("base", "t4"):
    setv(v)
    fr = L.compress_frame(src, sd)
    dig[v] = (fr.numel(), L.xxh32(fr))
    del fr
print("8 GiB B4 frames:", dig, "identical" if dig["base"] == dig["t4"] else "DIFFER", flush=True)
L.lib.lz4mtHipSetTiming(1)
ms = (ctypes.c_float * 4)()
for rep in range(3):
    for v in ("base", "t4"):
        setv(v)
        torch.cuda.synchronize()
        fr = L.compress_frame(src, sd)
        torch.cuda.synchronize()
        L.lib.lz4mtHipGetTimings(ms)
        print(f"pass {rep} {v}: encode {ms[0]:.2f} ms", flush=True)
        del fr
sys.exit(1 if bad or dig["base"] != dig["t4"] else 0)
