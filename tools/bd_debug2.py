"""-BD encode debug: does the memory before the input change block 0?"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402
from conftest import bd_input, read_golden  # noqa: E402

g = json.load(open(os.path.join(ROOT, "tests/golden/golden.json")))
f = g["bd_frames"][0]
data = bd_input(f["bytes"], f["seed"])
gold = read_golden(f["file"])
sd = L.make_sd(f["bid"], f["stream_checksum"], f["block_checksum"], block_dependence=True)
src = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
for fill in (0, 0x41, 0xFF, None):
    buf = torch.empty(len(data) + (1 << 20), dtype=torch.uint8, device="cuda")
    if fill is None:
        buf.random_(0, 256)
    else:
        buf.fill_(fill)
    t = buf[1 << 20:]
    t.copy_(src)
    out = bytes(L.compress_frame(t, sd).cpu().numpy().tobytes())
    print("fill", fill, "match gold", out == gold, len(out), len(gold), out[7:13].hex(), flush=True)
    os.environ["LZ4MT_AMD_BD_SERIAL"] = "1"
    out = bytes(L.compress_frame(t, sd).cpu().numpy().tobytes())
    del os.environ["LZ4MT_AMD_BD_SERIAL"]
    print("  serial match gold", out == gold, len(out), flush=True)
print("indep", len(bytes(L.compress_frame(src, L.make_sd(4, False, True)).cpu().numpy().tobytes())))
