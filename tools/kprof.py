"""One compress + decompress of N GiB (default 2) for PMC profiling."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
n = int(gib * (1 << 30))
src = L.gen_synthetic(n)
sd = L.make_sd(7, False, True)
fr = L.compress_frame(src, sd)
out, r = L.decompress_frame(fr)
torch.cuda.synchronize()
assert r == 0 and torch.equal(out, src)
print("ok", n, fr.numel())
