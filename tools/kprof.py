"""One compress + decompress of N GiB (default 8) for PMC profiling
(--bid K: block maximum size id K, default 7 = 4 MiB).
--random: splitmix64 bytes instead of App. F (every block stored raw): the
encoder then streams its source exactly once and the decoder copies raw
blocks, so FETCH_SIZE of those launches is measured against a known byte
count (the calibration tools/pmcsum.py records)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
gib = float(args[0]) if args else 8.0
n = int(gib * (1 << 30))
if "--random" in sys.argv:
    g = torch.Generator(device="cuda").manual_seed(5)
    src = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
else:
    src = L.gen_synthetic(n)
bid = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--bid=")), 7))
sd = L.make_sd(bid, False, True)
fr = L.compress_frame(src, sd)
out, r = L.decompress_frame(fr)
torch.cuda.synchronize()
assert r == 0 and torch.equal(out, src)
print("ok", n, fr.numel())
