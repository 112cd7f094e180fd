"""Does the encoder end on a tail?  k_encode time (the product kernel, timed
by the library's HIP events) on 8 GiB of 4 MiB blocks: the App. F input
itself, and 2048 copies of one of its blocks -- the median-cost, the
fastest and the slowest block by the diagnostic twin's per-block cycles
(tools/blockspread.py).  With identical blocks every wave does the same
work, so (real - median copies) is what the spread costs.
usage: python tools/tail_probe.py [block_id]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402

bid = int(sys.argv[1]) if len(sys.argv) > 1 else 7
bm = 1 << (8 + 2 * bid)
n = (8 << 30) // bm * bm
nb = n // bm
src = L.gen_synthetic(n)
torch.cuda.synchronize()
buf = (ctypes.c_uint64 * (nb * 16))()
assert L.lib.lz4mtHipDebugEncodeBlockStats(ctypes.c_void_p(src.data_ptr()), n, bm, buf, None) == 0
cyc = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 16)[:, :10].sum(axis=1).astype(np.float64)
order = np.argsort(cyc)
picks = {"median": int(order[nb // 2]), "fastest": int(order[0]), "slowest": int(order[-1]),
         "p90": int(order[int(nb * 0.9)])}
sd = L.make_sd(bid, False, True)
L.lib.lz4mtHipSetTiming(1)
ms = (ctypes.c_float * 4)()


def enc_ms(x):
    best = 1e9
    for _ in range(3):
        fr = L.compress_frame(x, sd)
        torch.cuda.synchronize()
        L.lib.lz4mtHipGetTimings(ms)
        best = min(best, ms[0])
        del fr
    return best


print(f"B{bid}, {nb} blocks; per-block cycles (twin) max/mean {cyc.max() / cyc.mean():.4f}, std/mean {cyc.std() / cyc.mean():.4f}")
print(f"  App. F input: k_encode {enc_ms(src):.2f} ms")
blocks = src.view(nb, bm)
for name, b in picks.items():
    rep = blocks[b].repeat(nb)
    torch.cuda.synchronize()
    print(f"  {nb} copies of block {b} ({name}, {cyc[b] / cyc.mean():.3f} of the mean): k_encode {enc_ms(rep):.2f} ms")
    del rep
# the same blocks, heaviest first (dispatch order = block order)
perm = torch.from_numpy(order[::-1].copy()).cuda()
srt = blocks[perm].reshape(-1)
torch.cuda.synchronize()
print(f"  App. F blocks sorted heaviest first: k_encode {enc_ms(srt):.2f} ms")
