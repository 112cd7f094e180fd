"""Encode-kernel time only (8 GiB App. F, BID 7 unless BID=..; best of 3), for timing
experiments whose output is not a valid frame: LZ4MT_AMD_LIB=<variant .so> python tools/enc_only.py"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402

src = L.gen_synthetic(8 << 30)
sd = L.make_sd(int(os.environ.get("BID", "7")), False, True)
L.lib.lz4mtHipSetTiming(1)
ms = (ctypes.c_float * 4)()
enc = 1e9
for _ in range(3):
    fr = L.compress_frame(src, sd)
    torch.cuda.synchronize()
    L.lib.lz4mtHipGetTimings(ms)
    enc = min(enc, ms[0])
    del fr
print(f"{os.path.basename(os.environ.get('LZ4MT_AMD_LIB', 'product'))}: encode {enc:.2f} ms (encode only)")
