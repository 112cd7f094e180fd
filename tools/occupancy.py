"""Encode/decode kernel time vs number of 4 MiB blocks (64 .. 2048): separates
per-wave latency (flat per-block time) from contention (time grows with load)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402

bm = 4 << 20
sd = L.make_sd(7, False, True)
L.lib.lz4mtHipSetTiming(1)
ms = (ctypes.c_float * 4)()
for nb in [int(a) for a in (sys.argv[1:] or ["64", "256", "512", "1024", "2048"])]:
    n = nb * bm
    src = L.gen_synthetic(n)
    enc, dec = [], []
    for _ in range(3):
        fr = L.compress_frame(src, sd)
        L.lib.lz4mtHipGetTimings(ms)
        enc.append(ms[0])
        out, r = L.decompress_frame(fr)
        L.lib.lz4mtHipGetTimings(ms)
        dec.append(ms[1])
    assert torch.equal(out, src)
    print(f"blocks {nb:5d}: encode {min(enc):8.2f} ms  decode {min(dec):7.2f} ms  "
          f"(per-CU waves {nb/256:.2f})", flush=True)
    del src, fr, out
    torch.cuda.empty_cache()
