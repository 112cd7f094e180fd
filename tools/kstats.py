"""Per-phase cycle breakdown of the encode/decode kernels (diagnostic twins).

usage: python tools/kstats.py [GiB] [block_id]
"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
bid = int(sys.argv[2]) if len(sys.argv) > 2 else 7
bm = 1 << (8 + 2 * bid)
n = int(gib * (1 << 30)) // bm * bm
src = L.gen_synthetic(n)
torch.cuda.synchronize()
st16 = (ctypes.c_uint64 * 16)()
t = time.time()
assert L.lib.lz4mtHipDebugEncodeStats(ctypes.c_void_p(src.data_ptr()), n, bm, st16, None) == 0
wall = time.time() - t
e = list(st16)
nb = n // bm
# encode_block_v5 phases (4 MiB .. 65547 B blocks)
names = ["probe", "stop+round trip", "table writes", "back+count", "layout", "-", "-", "-", "-", "-"]
tot = sum(e[:10])
names[5] = "(loop top)"
win = max(e[10], 1)
print(f"ENCODE {gib} GiB B{bid}: wall {wall*1e3:.1f} ms, blocks {nb}, windows {e[10]}, cycles/block {tot/nb:.3e}, "
      f"tag aliases {e[11]}, predecessor resolutions {e[12]}, wide windows {e[13]}")
for i in range(10):
    print(f"  {names[i]:14s} {e[i]/tot*100:5.1f}%  {e[i]/win:8.1f} cyc/window")
sd = L.make_sd(bid, False, True)
fr = L.compress_frame(src, sd)
torch.cuda.synchronize()
dst16 = (ctypes.c_uint64 * 16)()
t = time.time()
assert L.lib.lz4mtHipDebugDecodeStats(ctypes.c_void_p(fr.data_ptr()), fr.numel(), dst16, None) == 0
wall = time.time() - t
d = list(dst16)
print(f"DECODE: wall {wall*1e3:.1f} ms (incl. walk+alloc), total cycles/block {d[5]/nb:.3e}, batches {d[4]}, "
      f"sequences {d[6]} (batch {d[8]}, serial {d[9]}), far {d[7]} ({d[7]/max(d[6],1)*100:.1f}%)")
dn = ["between batches", "group copy", "ordered matches", "longlit+far write"]
for i in range(4):
    print(f"  {dn[i]:16s} {d[i]/d[5]*100:5.1f}%  {d[i]/max(d[6],1):8.1f} cyc/seq")
bn = {10: "refill", 11: "deltas", 12: "hop", 13: "fields+scan+check", 14: "flush", 15: "far issue"}
for i in range(10, 16):
    print(f"  {bn[i]:16s} {d[i]/d[5]*100:5.1f}%  {d[i]/max(d[4],1):8.1f} cyc/batch")
