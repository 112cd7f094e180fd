"""What the root still does after the encodes end in the streamed gather
(dist.compress_gather_streamed), measured on ONE GPU in one process: the
exposed tail of the 8-GPU compress that no single-GPU run shows.

  1. encode an 8 GiB App. F shard with publishing (lz4mtHipShardEncode);
  2. one non-final round afterwards takes everything published (what the
     rounds during the encode would have moved), then the FINAL round: the
     block tails since each block's last publish, stored sizes, checksums --
     the pack a sender pushes after its encode, timed (plan + pack) with its
     bytes reported;
  3. unpack of that final pack into a mirror, timed;
  4. the root's assembly of W shard bodies from mirrors (W = 8: 8 x 4.24 GB
     into one frame), timed -- the copy the root cannot start before every
     shard's sizes are known.
usage: python tools/tail_model.py [GiB per shard] [W]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402
from lz4mt_amd import dist as D  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
W = int(sys.argv[2]) if len(sys.argv) > 2 else 8
n = int(gib * (1 << 30)) // (4 << 20) * (4 << 20)
sd = L.make_sd(7, False, True)
src = L.gen_synthetic(n)
ws = L.shard_workspace(n, sd)
cap = 128 << 10
pack = torch.empty(L.shard_pack_bound(n, sd, 4 << 20), dtype=torch.uint8, device="cuda")
mirror = L.shard_workspace(n, sd)


def ms(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3, r


L.shard_reset(n, sd, ws)
t_enc, _ = ms(lambda: L.shard_encode(src, sd, ws))
# everything published during the encode (cap = the block size: one round)
_, _ = ms(lambda: L.shard_pack(src, sd, ws, pack, 4 << 20, False))
hdr = D.parse_pack_header(pack[:64].cpu().numpy().tobytes())
pub_bytes = hdr[1]
L.shard_unpack(pack, n, sd, mirror)
# the final round: tails + sizes + checksums
t_pack, _ = ms(lambda: L.shard_pack(src, sd, ws, pack, cap, True))
fin = D.parse_pack_header(pack[:64].cpu().numpy().tobytes())
t_unpack, _ = ms(lambda: L.shard_unpack(pack, n, sd, mirror))
body = L.shard_body_bytes(n, sd, mirror)
frame = torch.empty(W * body + 64, dtype=torch.uint8, device="cuda")


def assemble_all():
    for w in range(W):
        L.shard_assemble(None, n, sd, mirror, frame[w * body:(w + 1) * body])


t_asm, _ = ms(assemble_all)
t_asm2, _ = ms(assemble_all)
ref = L.compress_frame(src, sd)
ok = torch.equal(frame[:body], ref[7:7 + body])
print(f"shard {n >> 20} MiB: encode+xxh32 {t_enc:.1f} ms; published during the encode {pub_bytes / 1e6:.1f} MB of "
      f"{body / 1e6:.1f} MB records")
print(f"final round: {fin[1] / 1e6:.2f} MB payload ({fin[0] / 1e6:.2f} MB pack), plan+pack {t_pack:.2f} ms, "
      f"unpack {t_unpack:.2f} ms, complete={fin[2]}")
print(f"root assembly of {W} shard bodies ({W * body / 1e9:.2f} GB): {t_asm:.2f} / {t_asm2:.2f} ms; "
      f"body == single-process frame's records: {ok}")
