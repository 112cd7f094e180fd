"""Encode-kernel time only (8 GiB, 4 MiB blocks) for A/B timing of experiment
builds: LZ4MT_AMD_LIB=<variant .so> python tools/enc_time.py"""
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
best = 1e9
for _ in range(3):
    L.compress_frame(src, sd)
    L.lib.lz4mtHipGetTimings(ms)
    best = min(best, ms[0])
print(f"{os.path.basename(os.environ.get('LZ4MT_AMD_LIB', 'product'))}: encode {best:.2f} ms")
