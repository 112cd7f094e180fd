"""HC encode kernel time (8 GiB App. F, 4 MiB blocks, levels HC_LEVELS = 3,9,10,12; best of 2) for A/B of
experiment builds: LZ4MT_AMD_LIB=<variant .so> python tools/hctime.py"""
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
res = []
for level in (int(v) for v in os.environ.get("HC_LEVELS", "3,9,10,12").split(",")):
    best, size = 1e9, 0
    for _ in range(2):
        fr = L.compress_frame(src, sd, level=level)
        torch.cuda.synchronize()
        L.lib.lz4mtHipGetTimings(ms)
        best, size = min(best, ms[0]), fr.numel()
        del fr
    res.append(f"level {level}: encode {best:.1f} ms, frame {size}")
print(os.path.basename(os.environ.get("LZ4MT_AMD_LIB", "product")) + ": " + "; ".join(res), flush=True)
