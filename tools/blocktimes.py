"""Per-block start / end times of the product k_encode (an experiment build,
LZ4MT_EXP_BLKTIME: wall clock at 100 MHz, and each wave's HW_ID / XCC_ID):
how long the kernel runs after the average block is done, and whether the
late blocks share SIMDs / CUs / XCDs.
usage: LZ4MT_AMD_LIB=exp_libs/blktime.so python tools/blocktimes.py [block_id] [--sorted] [--decode]
(--decode: the same for k_decode, decompressing the frame)"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402

bid = int(next((a for a in sys.argv[1:] if not a.startswith("-")), 7))
bm = 1 << (8 + 2 * bid)
n = (8 << 30) // bm * bm
nb = n // bm
src = L.gen_synthetic(n)
if "--sorted" in sys.argv:   # heaviest first by the twin's per-block cycles
    buf = (ctypes.c_uint64 * (nb * 16))()
    assert L.lib.lz4mtHipDebugEncodeBlockStats(ctypes.c_void_p(src.data_ptr()), n, bm, buf, None) == 0
    cyc = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 16)[:, :10].sum(axis=1)
    src = src.view(nb, bm)[torch.from_numpy(np.argsort(-cyc).copy()).cuda()].reshape(-1).contiguous()
raw = ctypes.CDLL(os.environ["LZ4MT_AMD_LIB"])
raw.lz4mtHipExpBlockTimes.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
sd = L.make_sd(bid, False, True)
L.lib.lz4mtHipSetTiming(1)
ms = (ctypes.c_float * 4)()
dec = "--decode" in sys.argv
raw.lz4mtHipExpDecBlockTimes.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
frame = L.compress_frame(src, sd) if dec else None
for rep in range(3):
    if dec:
        fr, r = L.decompress_frame(frame)
        torch.cuda.synchronize()
        assert r == 0
        L.lib.lz4mtHipGetTimings(ms)
        ms[0] = ms[1]   # the decode kernel's time
    else:
        fr = L.compress_frame(src, sd)
        torch.cuda.synchronize()
        L.lib.lz4mtHipGetTimings(ms)
    out = np.zeros(nb * 3, dtype=np.uint64)
    assert (raw.lz4mtHipExpDecBlockTimes if dec else raw.lz4mtHipExpBlockTimes)(out.ctypes.data, nb) == nb
    t = out.reshape(nb, 3)
    t0, t1, hw = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64), t[:, 2]
    start = (t0 - t0.min()) / 1e5   # ms (100 MHz)
    end = (t1 - t0.min()) / 1e5
    dur = end - start
    print(f"B{bid} pass {rep}: {'k_decode' if dec else 'k_encode'} {ms[0]:.2f} ms; block end mean {end.mean():.2f} ms, p50 {np.median(end):.2f}, "
          f"p90 {np.percentile(end, 90):.2f}, max {end.max():.2f}; start spread {start.max():.2f} ms; "
          f"duration min {dur.min():.2f} mean {dur.mean():.2f} max {dur.max():.2f}")
    del fr
hwid = (hw & 0xFFFFFFFF).astype(np.int64)
xcc = (hw >> 32).astype(np.int64) & 0xF
simd = (hwid >> 4) & 3
cu = (hwid >> 8) & 15
sh = (hwid >> 12) & 1
se = (hwid >> 13) & 7
slot = hwid & 15
key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
print(f"  placement: {len(np.unique(xcc))} XCCs, {len(np.unique(key))} CUs, waves per CU max {np.bincount(key).max()}")
late = np.argsort(-end)[:16]
print("  latest blocks (block: end ms, duration, xcc/se/sh/cu/simd/slot):")
for b in late:
    print(f"    {b}: {end[b]:.2f} {dur[b]:.2f}  {xcc[b]}/{se[b]}/{sh[b]}/{cu[b]}/{simd[b]}/{slot[b]}")
for sl in np.unique(slot):
    m = slot == sl
    print(f"  wave slot {sl}: {m.sum()} blocks, end mean {end[m].mean():.2f} ms, max {end[m].max():.2f}")
out_dir = os.environ.get("BT_OUT")
if out_dir:
    tag = os.path.basename(os.environ["LZ4MT_AMD_LIB"]).split(".")[0]
    np.savez(os.path.join(out_dir, f"bt_{tag}_b{bid}{'_sorted' if '--sorted' in sys.argv else ''}{'_dec' if dec else ''}.npz"),
             start=start, end=end, xcc=xcc, se=se, sh=sh, cu=cu, simd=simd, slot=slot)
simdkey = key * 4 + simd
_, inv, cnt = np.unique(simdkey, return_inverse=True, return_counts=True)
pair_end = np.zeros(cnt.size)
np.maximum.at(pair_end, inv, end)
print(f"  waves per SIMD: {np.bincount(cnt)}; SIMD finish mean {pair_end.mean():.2f} ms, max {pair_end.max():.2f}")
xend = [end[xcc == x].max() for x in np.unique(xcc)]
print("  XCC finish: " + " ".join(f"{v:.1f}" for v in xend))
