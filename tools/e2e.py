"""End-to-end (PCIe-inclusive) rate of the reference-shaped API: lz4mtCompress /
lz4mtDecompress in LZ4MT_MODE_DEVICE over host memory (Lz4MtMemIo callbacks:
one read() per block into pinned staging, H2D, kernels, D2H, in-order write()).
With --file the same runs go file -> file through the FILE* callbacks
(lz4mtIoBindCstdio, the reference's src/lz4mt_io_cstdio.cpp path); the files
sit in the page cache (written just before), so this is the host-memory-speed
case of the file path.
Memory runs: best of 3 after a warm-up (E2E_REPS).
usage: python tools/e2e.py [GiB] [block_id] [--file DIR]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import lz4mt_amd as L  # noqa: E402
from lz4mt_amd import _abi  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
fdir = sys.argv[sys.argv.index("--file") + 1] if "--file" in sys.argv else None
if fdir:
    args = [a for a in args if a != fdir]
gib = float(args[0]) if len(args) > 0 else 2.0
bid = int(args[1]) if len(args) > 1 else 7
n = int(gib * (1 << 30))
REPS = int(os.environ.get("E2E_REPS", "3"))
src = L.gen_synthetic(n).cpu().numpy()
frame = np.empty(n + n // 1000 + (1 << 20), dtype=np.uint8)
out = np.empty(n + 64, dtype=np.uint8)


def run_mem(fn, inp, in_len, outp, out_cap, sd, mode):
    io = _abi.Lz4MtMemIo(inp.ctypes.data, in_len, 0, 0, outp.ctypes.data, out_cap, 0)
    ctx = L.init_context()
    ctx.mode = mode
    L.lib.lz4mtMemBind(ctypes.byref(ctx), ctypes.byref(io))
    t = time.perf_counter()
    r = fn(ctypes.byref(ctx), ctypes.byref(sd))
    return r, time.perf_counter() - t, io.outPos


def run_file(fn, path_in, path_out, sd, mode):
    ctx = L.init_context()
    ctx.mode = mode
    L.lib.lz4mtIoBindCstdio(ctypes.byref(ctx))
    assert L.lib.lz4mtIoOpenIstream(ctypes.byref(ctx), path_in.encode())
    assert L.lib.lz4mtIoOpenOstream(ctypes.byref(ctx), path_out.encode(), 0)
    t = time.perf_counter()
    r = fn(ctypes.byref(ctx), ctypes.byref(sd))
    L.lib.lz4mtIoCloseIstream(ctypes.byref(ctx))
    L.lib.lz4mtIoCloseOstream(ctypes.byref(ctx))   # fclose: the last writes land in the page cache
    return r, time.perf_counter() - t, os.path.getsize(path_out)


if fdir:
    pin, pfr, pout = (os.path.join(fdir, f"e2e_{k}") for k in ("in.bin", "frame.lz4", "out.bin"))
    src.tofile(pin)
    # the file path's floor: writing n bytes into a fresh file of this
    # filesystem from host memory, one thread (fwrite-like) and 8 threads
    # (pwrite at disjoint offsets), and reading it back
    import concurrent.futures as cf
    pw = os.path.join(fdir, "e2e_wr.bin")
    for rep in range(2):
        if os.path.exists(pw):
            os.remove(pw)
        t = time.perf_counter()
        src.tofile(pw)
        w1 = n / (time.perf_counter() - t) / 2**30
        os.remove(pw)
        fd = os.open(pw, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        mv = memoryview(src).cast("B")
        step = -(-n // 8)
        t = time.perf_counter()
        with cf.ThreadPoolExecutor(8) as ex:
            list(ex.map(lambda i: os.pwrite(fd, mv[i * step:min(n, (i + 1) * step)], i * step), range(8)))
        w8 = n / (time.perf_counter() - t) / 2**30
        os.close(fd)
        t = time.perf_counter()
        back = np.fromfile(pw, dtype=np.uint8)
        r1 = n / (time.perf_counter() - t) / 2**30
        del back
        print(f"floor {gib:g} GiB into {fdir}: write 1 thread {w1:.2f} GiB/s, 8 threads {w8:.2f} GiB/s, "
              f"read back {r1:.2f} GiB/s", flush=True)
    os.remove(pw)
for label, sck in (("-Sx -BX", False), ("default flags (serial stream XXH32 on the host)", True)):
    sd = L.make_sd(bid, stream_checksum=sck, block_checksum=not sck)
    sdo = L.init_stream_descriptor()
    if fdir:
        run_file(L.lib.lz4mtCompress, pin, pfr, sd, L.MODE_DEVICE)   # warm-up
        r, tc, flen = run_file(L.lib.lz4mtCompress, pin, pfr, sd, L.MODE_DEVICE)
        assert r == 0, r
        run_file(L.lib.lz4mtDecompress, pfr, pout, sdo, L.MODE_DEVICE)
        r, td, olen = run_file(L.lib.lz4mtDecompress, pfr, pout, sdo, L.MODE_DEVICE)
        assert r == 0 and olen == n and np.array_equal(np.fromfile(pout, dtype=np.uint8), src), (r, olen)
        where = "file -> GPU -> file, page cache"
    else:
        run_mem(L.lib.lz4mtCompress, src, n, frame, frame.size, sd, L.MODE_DEVICE)   # warm-up
        tc = td = 1e9
        for _ in range(REPS):   # best of REPS (host memory bandwidth varies from run to run)
            r, t_, flen = run_mem(L.lib.lz4mtCompress, src, n, frame, frame.size, sd, L.MODE_DEVICE)
            assert r == 0, r
            tc = min(tc, t_)
        run_mem(L.lib.lz4mtDecompress, frame, flen, out, out.size, sdo, L.MODE_DEVICE)   # warm-up
        for _ in range(REPS):
            r, t_, olen = run_mem(L.lib.lz4mtDecompress, frame, flen, out, out.size, sdo, L.MODE_DEVICE)
            td = min(td, t_)
        assert os.environ.get("E2E_NOCHECK") == "1" or (r == 0 and olen == n and np.array_equal(out[:n], src)), (r, olen)
        where = "host memory -> GPU -> host memory"
    print(f"e2e {gib:g} GiB B{bid} {label}: compress {n / tc / 2**30:.2f} GiB/s, "
          f"decompress {n / td / 2**30:.2f} GiB/s ({where}, ratio {n / flen:.3f})", flush=True)
if fdir:
    for p in (pin, pfr, pout):
        os.remove(p)
