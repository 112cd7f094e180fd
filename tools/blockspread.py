"""Spread of the encoder's per-block cost (diagnostic twin k_encode_stats):
with exactly one generation of waves (8 GiB of 4 MiB blocks at 8 waves per
CU) the slowest block sets the kernel time, so max / mean of the per-block
cycles bounds what balancing could buy.
usage: python tools/blockspread.py [GiB] [block_id]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
bid = int(sys.argv[2]) if len(sys.argv) > 2 else 7
bm = 1 << (8 + 2 * bid)
n = int(gib * (1 << 30)) // bm * bm
nb = n // bm
src = L.gen_synthetic(n)
torch.cuda.synchronize()
buf = (ctypes.c_uint64 * (nb * 16))()
assert L.lib.lz4mtHipDebugEncodeBlockStats(ctypes.c_void_p(src.data_ptr()), n, bm, buf, None) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 16).astype(np.float64)
cyc = a[:, :10].sum(axis=1)
win = a[:, 10]
q = np.percentile(cyc, [0, 1, 10, 50, 90, 99, 100])
print(f"{gib} GiB B{bid}: {nb} blocks; cycles per block mean {cyc.mean():.4e}, max/mean {cyc.max() / cyc.mean():.4f}, "
      f"min/mean {cyc.min() / cyc.mean():.4f}, std/mean {cyc.std() / cyc.mean():.4f}")
print("  percentiles 0/1/10/50/90/99/100 of cycles / mean: " + " ".join(f"{x / cyc.mean():.4f}" for x in q))
print(f"  windows per block mean {win.mean():.0f}, max/mean {win.max() / win.mean():.4f}; "
      f"corr(cycles, windows) {np.corrcoef(cyc, win)[0, 1]:.3f}")
top = np.argsort(-cyc)[:8]
print("  slowest blocks: " + ", ".join(f"{i} ({cyc[i] / cyc.mean():.3f})" for i in top))
