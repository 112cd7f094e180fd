"""Encoder time per 8 GiB of App. F against block (= stream) size and
resident waves per CU, for the split-parse A/B.

lz4mtHipDebugEncode runs the frame path's block encoder over blocks of ANY
size (512 KiB and 2 MiB too: the streams of a 4 MiB block split in 8 or 2);
LZ4MT_AMD_ENC picks k_encode (4096 x u32 table, 20 KiB LDS, 8 waves/CU) or
k_encode_p17 (3-byte table, 14.25 KiB, 11 waves/CU); LZ4MT_AMD_ENC_LDS_PAD
adds dynamic LDS to the launch, i.e. fewer resident waves.  A split parse
of 4 MiB blocks into streams of S bytes costs about (time at S) x (1 +
overlap / S) plus the joins, so these rows bound what it can gain.
Timing: HIP events on the launch stream, best of 3.
--overlap: instead, time the split parse's parse work directly
(lz4mtHipDebugEncodeOverlap: stream b of S bytes parsed cold from ov bytes
before its start, the overlap its join needs; 410 KiB = the mean measured
by tools/split_sim.py, 1018 KiB = its maximum), joins not included.
usage: python tools/occ_sweep.py [--overlap]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402

LDS_CU = 163840
STATIC = {"base": 20480, "p17": 14592}   # static LDS of k_encode (ENCODE_LDS) and k_encode_p17 (PLDS)
N = 8 << 30
src = L.gen_synthetic(N)
slots = torch.empty(N + (8 << 20), dtype=torch.uint8, device="cuda")
csize = torch.empty(N // 65536 + 64, dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream()


def run(bs, enc, waves=None):
    os.environ["LZ4MT_AMD_ENC"] = enc
    pad = max(0, LDS_CU // waves - STATIC[enc]) if waves else 0
    os.environ["LZ4MT_AMD_ENC_LDS_PAD"] = str(pad)
    best = 1e9
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        if L.lib.lz4mtHipDebugEncode(ctypes.c_void_p(src.data_ptr()), N, bs, ctypes.c_void_p(slots.data_ptr()),
                                     ctypes.c_void_p(csize.data_ptr()), ctypes.c_void_p(st.cuda_stream)) != 0:
            raise RuntimeError("lz4mtHipDebugEncode")
        b.record(st)
        b.synchronize()
        best = min(best, a.elapsed_time(b))
    nb = N // bs
    total = int(csize[:nb].clamp(min=0).sum().item())
    return best, pad, total




def run_overlap(S, ov, enc):
    nb = (N + S - 1) // S
    out = torch.empty(nb * (S + ov) + 64, dtype=torch.uint8, device="cuda")
    cs = torch.empty(nb, dtype=torch.int32, device="cuda")
    best = 1e9
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        if L.lib.lz4mtHipDebugEncodeOverlap(ctypes.c_void_p(src.data_ptr()), N, S, ov, int(enc == "p17"),
                                            ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(cs.data_ptr()),
                                            ctypes.c_void_p(st.cuda_stream)) != 0:
            raise RuntimeError("lz4mtHipDebugEncodeOverlap")
        b.record(st)
        b.synchronize()
        best = min(best, a.elapsed_time(b))
    bad = int((cs <= 0).sum().item())
    del out
    return best, bad


if "--overlap" in sys.argv:
    print("split parse, parse work only: stream S, overlap ov, encoder: ms per 8 GiB", flush=True)
    for S in (512 << 10, 1 << 20, 2 << 20):
        for ov in (0, 410 << 10, 1018 << 10):
            for enc in ("base", "p17"):
                t, bad = run_overlap(S, ov, enc)
                print(f"S {S >> 10:5d} KiB ov {ov >> 10:5d} KiB {enc:4s}: {t:8.2f} ms"
                      + (f"  ({bad} streams raw/failed)" if bad else ""), flush=True)
    sys.exit(0)

print("stream/block size, encoder, waves/CU (LDS pad): encode ms per 8 GiB, encoded bytes", flush=True)
for bs in (256 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20):
    for enc in ("base", "p17"):
        t, _, tot = run(bs, enc)
        print(f"{bs >> 10:5d} KiB {enc:4s} full occupancy: {t:8.2f} ms  ({tot} B)", flush=True)
for bs in (512 << 10, 1 << 20):
    for enc, waves in (("base", (7, 6, 5, 4)), ("p17", (10, 9, 8, 6))):
        for w in waves:
            t, pad, _ = run(bs, enc, w)
            print(f"{bs >> 10:5d} KiB {enc:4s} waves/CU {w:2d} (pad {pad:5d} B): {t:8.2f} ms", flush=True)
os.environ.pop("LZ4MT_AMD_ENC_LDS_PAD")
os.environ.pop("LZ4MT_AMD_ENC")
