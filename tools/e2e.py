"""End-to-end (PCIe-inclusive) rate of the reference-shaped API: lz4mtCompress /
lz4mtDecompress in LZ4MT_MODE_DEVICE over host memory (Lz4MtMemIo callbacks:
one read() per block into pinned staging, H2D, kernels, D2H, in-order write()).
usage: python tools/e2e.py [GiB] [block_id]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402
from lz4mt_amd import _abi  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
bid = int(sys.argv[2]) if len(sys.argv) > 2 else 7
n = int(gib * (1 << 30))
src = L.gen_synthetic(n).cpu().numpy()
frame = np.empty(n + n // 1000 + (1 << 20), dtype=np.uint8)
out = np.empty(n + 64, dtype=np.uint8)


def run(fn, inp, in_len, outp, out_cap, sd, mode):
    io = _abi.Lz4MtMemIo(inp.ctypes.data, in_len, 0, 0, outp.ctypes.data, out_cap, 0)
    ctx = L.init_context()
    ctx.mode = mode
    L.lib.lz4mtMemBind(ctypes.byref(ctx), ctypes.byref(io))
    t = time.perf_counter()
    r = fn(ctypes.byref(ctx), ctypes.byref(sd))
    return r, time.perf_counter() - t, io.outPos


for label, sck in (("-Sx -BX", False), ("default flags (serial stream XXH32 on the host)", True)):
    sd = L.make_sd(bid, stream_checksum=sck, block_checksum=not sck)
    run(L.lib.lz4mtCompress, src, n, frame, frame.size, sd, L.MODE_DEVICE)   # warm-up
    r, tc, flen = run(L.lib.lz4mtCompress, src, n, frame, frame.size, sd, L.MODE_DEVICE)
    assert r == 0, r
    sdo = L.init_stream_descriptor()
    run(L.lib.lz4mtDecompress, frame, flen, out, out.size, sdo, L.MODE_DEVICE)   # warm-up
    r, td, olen = run(L.lib.lz4mtDecompress, frame, flen, out, out.size, sdo, L.MODE_DEVICE)
    assert r == 0 and olen == n and np.array_equal(out[:n], src), (r, olen)
    print(f"e2e {gib:g} GiB B{bid} {label}: compress {n / tc / 2**30:.2f} GiB/s, "
          f"decompress {n / td / 2**30:.2f} GiB/s (host memory -> GPU -> host memory, ratio {n / flen:.3f})",
          flush=True)
