"""One warm end-to-end compress + decompress (host memory -> GPU -> host
memory, lz4mtCompress / lz4mtDecompress in LZ4MT_MODE_DEVICE, -Sx -BX) for a
profiler run: rocprofv3 --kernel-trace --memory-copy-trace -- python3 tools/e2e_one.py 8
(the second of two passes is the measured one; markers on stderr)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import lz4mt_amd as L  # noqa: E402
from lz4mt_amd import _abi  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
n = int(gib * (1 << 30))
src = L.gen_synthetic(n).cpu().numpy()
frame = np.empty(n + n // 1000 + (1 << 20), dtype=np.uint8)
out = np.empty(n + 64, dtype=np.uint8)
sd = L.make_sd(7, stream_checksum=False, block_checksum=True)


def run(fn, inp, in_len, outp, out_cap, sdx):
    io = _abi.Lz4MtMemIo(inp.ctypes.data, in_len, 0, 0, outp.ctypes.data, out_cap, 0)
    ctx = L.init_context()
    ctx.mode = L.MODE_DEVICE
    L.lib.lz4mtMemBind(ctypes.byref(ctx), ctypes.byref(io))
    t = time.perf_counter()
    r = fn(ctypes.byref(ctx), ctypes.byref(sdx))
    return r, time.perf_counter() - t, io.outPos


for rep in range(2):
    r, tc, flen = run(L.lib.lz4mtCompress, src, n, frame, frame.size, sd)
    assert r == 0, r
    sdo = L.init_stream_descriptor()
    r, td, olen = run(L.lib.lz4mtDecompress, frame, flen, out, out.size, sdo)
    assert r == 0 and olen == n, (r, olen)
    print(f"pass {rep}: compress {n / tc / 2**30:.2f} GiB/s ({tc * 1e3:.1f} ms), "
          f"decompress {n / td / 2**30:.2f} GiB/s ({td * 1e3:.1f} ms)", flush=True)
assert np.array_equal(out[:n], src)
