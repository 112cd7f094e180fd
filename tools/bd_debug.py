"""-BD encode: compare the parallel-round encoder with the serial kernel and
the golden frame block by block (debug aid)."""
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402
from conftest import bd_input, golden, read_golden  # noqa: E402,F401
import json  # noqa: E402

g = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests/golden/golden.json")))


def blocks(f, bck):
    pos, out = 7, []
    while True:
        w = struct.unpack_from("<I", f, pos)[0]
        pos += 4
        if w == 0:
            return out
        n = w & 0x7FFFFFFF
        out.append(f[pos - 4:pos + n + (4 if bck else 0)])
        pos += n + (4 if bck else 0)


for f in g["bd_frames"]:
    data = bd_input(f["bytes"], f["seed"])
    t = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    sd = L.make_sd(f["bid"], f["stream_checksum"], f["block_checksum"], block_dependence=True)
    par = bytes(L.compress_frame(t, sd).cpu().numpy().tobytes())
    os.environ["LZ4MT_AMD_BD_SERIAL"] = "1"
    ser = bytes(L.compress_frame(t, sd).cpu().numpy().tobytes())
    del os.environ["LZ4MT_AMD_BD_SERIAL"]
    gold = read_golden(f["file"])
    bp, bs, bg = blocks(par, f["block_checksum"]), blocks(ser, f["block_checksum"]), blocks(gold, f["block_checksum"])
    print(f["name"], "par==gold", par == gold, "ser==gold", ser == gold, "nblocks", len(bg),
          "par bad", [i for i in range(len(bg)) if i >= len(bp) or bp[i] != bg[i]][:20],
          "ser bad", [i for i in range(len(bg)) if i >= len(bs) or bs[i] != bg[i]][:20], flush=True)
    for name, fr in (("par", par), ("ser", ser)):
        i = next((k for k in range(min(len(fr), len(gold))) if fr[k] != gold[k]), None)
        print(" ", name, "len", len(fr), "gold", len(gold), "first diff at", i, fr[:12].hex(), gold[:12].hex(),
              "blk0", len(bp[0]) if name == "par" else len(bs[0]), len(bg[0]))
