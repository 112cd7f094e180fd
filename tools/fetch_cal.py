"""FETCH_SIZE calibration on a known byte count.

Run under `rocprofv3 --kernel-trace --pmc FETCH_SIZE` (and a second pass
with WRITE_SIZE if wanted): lz4mtHipDebugFetchCal reads N bytes exactly once
with 1-, 4-, 8- and 16-byte loads per lane (the encoder's byte loads, gld4u,
gld8u, and a dwordx4 stream), twice each, from a buffer that was just
overwritten (so its lines are not in any cache).  tools/pmcsum.py divides
each launch's FETCH_SIZE by N: the counted fraction for that load width,
accepted only if N / duration stays at or below the achievable HBM rate
(~6.3 TB/s, MI355X_MICROARCH.md).
usage: python tools/fetch_cal.py [GiB]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
n = int(gib * (1 << 30))
buf = torch.empty(n, dtype=torch.uint8, device="cuda")
flush = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
out = torch.zeros(1, dtype=torch.int32, device="cuda")
for width in (1, 4, 8, 16):
    for _ in range(2):
        buf.fill_(0x11 * width % 256)   # rewrite: nothing of it stays in L2 / MALL from a read
        flush.fill_(0)         # and push the tail of that write out of the caches
        torch.cuda.synchronize()
        assert L.lib.lz4mtHipDebugFetchCal(ctypes.c_void_p(buf.data_ptr()), n, width,
                                           ctypes.c_void_p(out.data_ptr()), None) == 0
        torch.cuda.synchronize()
print("ok", n)
