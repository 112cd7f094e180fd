"""Diagnostic of the fused walk + decode on a small frame (prints and exits)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402

data = L.gen_synthetic(3 << 20)
for bid in [int(a) for a in sys.argv[1:]] or (7, 6, 5, 4):
    fr = L.compress_frame(data, L.make_sd(bid, False, True))
    torch.cuda.synchronize()
    for mode in ("serial", "fused"):
        os.environ["LZ4MT_AMD_WALK"] = mode
        print(f"B{bid} {mode}: decoding", flush=True)
        t = time.perf_counter()
        out, r = L.decompress_frame(fr)
        print(f"B{bid} {mode}: returned after {(time.perf_counter() - t) * 1e3:.1f} ms", flush=True)
        torch.cuda.synchronize()
        print(f"B{bid} {mode}: r={r} equal={torch.equal(out, data)}", flush=True)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        out, r = L.decompress_frame(fr)
    s.synchronize()
    print(f"B{bid} fused on a torch stream: r={r} equal={torch.equal(out, data)}", flush=True)
