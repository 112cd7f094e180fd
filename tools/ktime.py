"""Encode and decode kernel times (8 GiB, 4 MiB blocks; best of 3) for A/B
timing of experiment builds: LZ4MT_AMD_LIB=<variant .so> python tools/ktime.py"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402

n = 8 << 30
src = L.gen_synthetic(n)
sd = L.make_sd(7, False, True)
L.lib.lz4mtHipSetTiming(1)
ms = (ctypes.c_float * 4)()
enc, dec = 1e9, 1e9
for _ in range(3):
    fr = L.compress_frame(src, sd)
    L.lib.lz4mtHipGetTimings(ms)
    enc = min(enc, ms[0])
    out, r = L.decompress_frame(fr)
    L.lib.lz4mtHipGetTimings(ms)
    dec = min(dec, ms[1])
    assert r == 0
    del fr, out
assert torch.equal(L.decompress_frame(L.compress_frame(src, sd))[0], src)
print(f"{os.path.basename(os.environ.get('LZ4MT_AMD_LIB', 'product'))}: encode {enc:.2f} ms  decode {dec:.2f} ms")
