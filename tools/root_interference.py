"""Does the root's own encode slow down while it unpacks the other ranks'
packs?  (The 8-GPU streamed gather, dist.compress_gather_streamed: the root
encodes its shard AND, every round, places up to 7 senders' packs into its
mirrors with k_shard_unpack -- LDS-free kernels that share the CUs with its
encoder waves.)  Measured on ONE GPU in one process:

  1. the root's encode alone: lz4mtHipShardEncode of an 8 GiB App. F shard
     (k_encode_pub + block checksums), HIP events on its stream;
  2. a real pack stream: the same shard packed in rounds of at most CAP bytes
     per block (what one sender pushes over its encode);
  3. the encode again while a second stream unpacks S senders' worth of those
     packs (S x the shard's records, into S mirrors), paced one round every
     ROUND_MS like the gather's rounds -- the root's load at 1 + S GPUs.
Each sender's stream is paced so that it spreads over the encode's length
(one round every encode_ms / packs), as in the real gather.
usage: python tools/root_interference.py [senders=7]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402
from lz4mt_amd import dist as D  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 7
n = 8 << 30
CAP = 32 << 10   # ~64 MiB per round: the gather's rounds of ~2-3 ms carry about that
sd = L.make_sd(7, False, True)
src = L.gen_synthetic(n)
ws = L.shard_workspace(n, sd)
enc = torch.cuda.Stream()
side = torch.cuda.Stream()


def encode_timed(during=None):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    L.shard_reset(n, sd, ws)
    enc.wait_stream(torch.cuda.current_stream())
    a.record(enc)
    L.shard_encode(src, sd, ws, stream=enc)
    b.record(enc)
    if during:
        during(b)
    b.synchronize()
    return a.elapsed_time(b)


t0 = encode_timed()
# a sender's pack stream over its encode: published bytes in rounds of <= CAP per block
L.shard_reset(n, sd, ws)
packs = []
buf = torch.empty(L.shard_pack_bound(n, sd, CAP), dtype=torch.uint8, device="cuda")
L.shard_encode(src, sd, ws)
torch.cuda.synchronize()
while True:
    L.shard_pack(src, sd, ws, buf, CAP, True)
    packed, payload, done, _ = D.parse_pack_header(buf[:64].cpu().numpy().tobytes())
    packs.append(buf[:packed].clone())
    if done:
        break
mirrors = [L.shard_workspace(n, sd) for _ in range(S)]
round_ms = t0 / len(packs)
print(f"encode alone {t0:.2f} ms; one sender's stream: {len(packs)} packs, "
      f"{sum(p.numel() for p in packs) / 1e9:.2f} GB", flush=True)


def unpack_all(end_ev):
    # one round every round_ms while the encode runs: each of the S senders'
    # next pack into its mirror (the packs repeat if the encode outlasts them)
    k = 0
    while not end_ev.query():
        t = time.perf_counter()
        with torch.cuda.stream(side):
            for s in range(S):
                L.shard_unpack(packs[k % len(packs)], n, sd, mirrors[s], stream=side)
        k += 1
        dt = round_ms * 1e-3 - (time.perf_counter() - t)
        if dt > 0:
            time.sleep(dt)
    side.synchronize()
    unpack_all.rounds = k


for rep in range(2):
    t1 = encode_timed(unpack_all)
    print(f"encode beside {S} senders' unpacks ({unpack_all.rounds} rounds, one every {round_ms:g} ms): "
          f"{t1:.2f} ms ({(t1 / t0 - 1) * 100:+.1f} %)", flush=True)
t2 = encode_timed()
print(f"encode alone again {t2:.2f} ms", flush=True)
