"""Encode and decode kernel times (8 GiB, 4 MiB blocks or BID=4..6; best of 3) for A/B
timing of experiment builds: LZ4MT_AMD_LIB=<variant .so> python tools/ktime.py"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402

n = 8 << 30
src = L.gen_synthetic(n)
sd = L.make_sd(int(os.environ.get("BID", "7")), False, os.environ.get("KTIME_BCK", "1") == "1")
L.lib.lz4mtHipSetTiming(1)
ms = (ctypes.c_float * 4)()
enc, dec, wc, wd, xc, xd = 1e9, 1e9, 1e9, 1e9, 1e9, 1e9
for _ in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fr = L.compress_frame(src, sd)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    L.lib.lz4mtHipGetTimings(ms)
    enc, xc = min(enc, ms[0]), min(xc, ms[1])
    out, r = L.decompress_frame(fr)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    wc, wd = min(wc, t1 - t0), min(wd, t2 - t1)
    L.lib.lz4mtHipGetTimings(ms)
    dec, xd = min(dec, ms[1]), min(xd, ms[2])
    assert r == 0 or os.environ.get("KTIME_NOCHECK") == "1"
    del fr, out
if os.environ.get("KTIME_NOCHECK") != "1":
    assert torch.equal(L.decompress_frame(L.compress_frame(src, sd))[0], src)
xcs = f"{xc:.2f}" if xc > 0.05 else "side stream"   # frame compress runs it beside the assembly
print(f"{os.path.basename(os.environ.get('LZ4MT_AMD_LIB', 'product'))}: encode {enc:.2f} ms  decode {dec:.2f} ms  "
      f"| block xxh32 {xcs} / {xd:.2f} ms (+verify) | compress call {wc * 1e3:.2f} ms  decompress call {wd * 1e3:.2f} ms")
