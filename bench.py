"""bench.py — device-resident LZ4 frame compress + decompress on MI355X.

Workload (BASELINE.json configs[1]): 8 GiB synthetic buffer per GPU
(SURVEY.md App. F generator), 4 MiB independent blocks, -Sx -BX frames
(block XXH32 on, serial content checksum off), compress + decompress +
XXH32, inputs resident in HBM when the timed region starts.  One step =
compress the buffer into one lz4mt frame, then decompress that frame (block
checksums verified by the decoder).  At N>1 each rank owns a contiguous
block range (its 8 GiB shard of the 8N GiB stream, weak scaling) and the
compressed shards are gathered to rank 0 over RCCL (the only exchange step
the path has); decompression is sharded with no collective.  The gather is
enqueued before the local decompress and runs over xGMI while each rank
decodes its own shard (both only read the compressed frame), so at N>1
compress_GiBps covers the encode and decompress_GiBps the decode + gather.

Prints ONE JSON line on rank 0 (value = uncompressed GiB of the whole job /
(compress + decompress time), plus the per-direction rates, the encode
kernel's roofline and the CPU baseline).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import lz4mt_amd as L  # noqa: E402
from lz4mt_amd import dist as D  # noqa: E402

GiB = float(1 << 30)
HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
GOLDEN = 0x9E3779B97F4A7C15


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--gib", type=float, default=8.0, help="GiB per GPU")
    p.add_argument("--block-id", type=int, default=7, help="4..7 = 64 KiB..4 MiB")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-mib", type=int, default=256, help="CPU baseline sample (MiB)")
    p.add_argument("--decompress-only", action="store_true",
                   help="configs[2]: time only the decompression of a pre-compressed stream (use --gib 32)")
    return p.parse_args()


def timings():
    ms = (ctypes.c_float * 4)()
    if L.lib.lz4mtHipGetTimings(ms) != 0:
        return None
    return list(ms)


def cpu_baseline(mib, block_id):
    """lz4mt-shaped CPU pipeline (oracle 'port'), bounded sample, rank 0 only."""
    import oracle
    n = mib << 20
    buf = ctypes.create_string_buffer(n)
    oracle.lib.orc_gen_synthetic(buf, n, 42)
    p = oracle.params(block_id, stream_checksum=False, block_checksum=True)
    threads = min(16, os.cpu_count() or 1)
    tc1, td1, fs = oracle.pipeline_roundtrip(buf, n, p, 1)
    tcN, tdN, _ = oracle.pipeline_roundtrip(buf, n, p, threads)
    return {
        "value": round(n / GiB / (tcN + tdN), 3), "unit": "GiB/s", "cores": threads, "kind": "port",
        "sample": f"{mib} MiB App.F synthetic, B{block_id} -Sx -BX, compress+decompress, lz4mt-shaped pipeline "
                  f"(nPool=threads+1, in-order writer) over the oracle codec",
        "compress_GiBps": round(n / GiB / tcN, 3), "decompress_GiBps": round(n / GiB / tdN, 3),
        "single_thread_compress_GiBps": round(n / GiB / tc1, 3),
        "single_thread_decompress_GiBps": round(n / GiB / td1, 3),
        "cpu_model": _cpu_model(),
    }


def pmc_traffic(kernel, n, bm):
    """HBM-side bytes per launch of `kernel` from the newest committed PMC
    summary (profiles/*_pmc.json, written by tools/prof.sh + tools/pmcsum.py on
    the same 8 GiB / 4 MiB-block workload); None when absent or not comparable."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")))   # round tags sort by name
    if not files or n != 8 << 30 or bm != 4 << 20:
        return None, None
    try:
        k = json.load(open(files[-1]))["kernels"][kernel]
    except (OSError, KeyError, ValueError):
        return None, None
    return k["fetch_bytes"] + k["write_bytes"], os.path.basename(files[-1])


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    stream = torch.cuda.current_stream()

    bm = 1 << (8 + 2 * a.block_id)
    n = int(a.gib * GiB) // bm * bm
    segs_per_rank = n // 65536
    seed = (42 + rank * segs_per_rank * GOLDEN) % (1 << 64)   # rank r = shard r of one global stream
    src = L.gen_synthetic(n, seed=seed, device=dev)
    sd = L.make_sd(a.block_id, stream_checksum=False, block_checksum=True)
    cap = L.frame_bound(n, sd)
    frame_buf = torch.empty(cap, dtype=torch.uint8, device=dev)
    ws = L.compress_workspace(n, sd, device=dev)
    out = torch.empty(n, dtype=torch.uint8, device=dev)
    fsz = torch.zeros(2, dtype=torch.int64, device=dev)

    def compress():
        r = L.lib.lz4mtHipCompressFrameAsync(
            ctypes.c_void_p(src.data_ptr()), n, ctypes.c_void_p(frame_buf.data_ptr()), cap,
            ctypes.c_void_p(fsz.data_ptr()), ctypes.byref(sd), ctypes.c_void_p(ws.data_ptr()), ws.numel(),
            ctypes.c_void_p(stream.cuda_stream))
        if r != 0:
            raise L.Lz4MtError(r, "compress")

    stitched = {"len": 0}

    def gather_to_root(flen):
        # one frame for the whole 8N GiB stream on rank 0 (lz4mt_amd/dist.py);
        # enqueued only: it runs over xGMI while this rank decodes its shard
        full, works = D.gather_frame(frame_buf, flen, dst=0, async_op=True)
        return full, works

    def decompress(flen):
        osz = ctypes.c_uint64(0)
        sdo = L.init_stream_descriptor()
        r = L.lib.lz4mtHipDecompressFrame(ctypes.c_void_p(frame_buf.data_ptr()), flen,
                                          ctypes.c_void_p(out.data_ptr()), out.numel(), ctypes.byref(osz),
                                          ctypes.byref(sdo), ctypes.c_void_p(stream.cuda_stream))
        if r != 0 or osz.value != n:
            raise L.Lz4MtError(r, f"decompress ({osz.value} of {n} bytes)")

    if a.decompress_only:   # compress once, untimed
        compress()
        torch.cuda.synchronize()
    L.lib.lz4mtHipSetTiming(1)
    tc = td = 0.0
    enc_ms, dec_ms, frame_len = [], [], 0
    for it in range(a.warmup + a.steps):
        timed = it >= a.warmup
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        tm = None
        if not a.decompress_only:
            compress()
        frame_len = int(fsz[0].item())          # synchronises the stream
        if not a.decompress_only:
            tm = timings()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        full, works = gather_to_root(frame_len) if world > 1 and not a.decompress_only else (None, [])
        decompress(frame_len)
        tmd = timings()
        for w in works:
            w.wait()
        if full is not None:
            stitched["len"] = full.numel()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t2 = time.perf_counter()
        if timed:
            tc += t1 - t0
            td += t2 - t1
            if tm:
                enc_ms.append(tm[0])
            if tmd:
                dec_ms.append(tmd[1])
    L.lib.lz4mtHipSetTiming(0)

    # correctness of the last step (not timed)
    ok = bool(torch.equal(out, src))
    if world > 1:
        t = torch.tensor([tc, td, 0.0 if ok else 1.0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        tc, td, bad = t.tolist()
        ok = bad == 0.0
    K = a.steps
    total = n * world * K
    comp_gibps = None if a.decompress_only else total / GiB / tc
    decomp_gibps = total / GiB / td
    value = decomp_gibps if a.decompress_only else total / GiB / (tc + td)

    enc_avg = sum(enc_ms) / len(enc_ms) if enc_ms else None
    dec_avg = sum(dec_ms) / len(dec_ms) if dec_ms else None
    body = frame_len - 7 - 4
    roof = None
    if enc_avg:
        alg = n + body                          # algorithmic bytes per encode launch
        ach = alg / (enc_avg * 1e-3) / 1e9
        traffic, tsrc = pmc_traffic("k_encode", n, bm)
        roof = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBPS, 5), "traffic": traffic, "kernel": "k_encode",
                "kernel_ms": round(enc_avg, 3), "algorithmic_bytes": alg,
                "traffic_source": f"profiles/{tsrc}: FETCH_SIZE + WRITE_SIZE per launch (raw counters)" if tsrc else None}
    dec_roof = None
    if dec_avg:
        alg = n + body
        ach = alg / (dec_avg * 1e-3) / 1e9
        dtraffic, _ = pmc_traffic("k_decode", n, bm)
        dec_roof = {"kernel": "k_decode", "kernel_ms": round(dec_avg, 3), "achieved": round(ach, 2),
                    "frac": round(ach / HBM_PEAK_GBPS, 5), "traffic": dtraffic}

    if a.decompress_only and dec_roof:   # the decode kernel is the dominant one here
        roof = {"bound": "hbm", "achieved": dec_roof["achieved"], "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": dec_roof["frac"], "traffic": dec_roof["traffic"], "kernel": "k_decode",
                "kernel_ms": dec_roof["kernel_ms"], "algorithmic_bytes": n + body}
    if rank == 0:
        cpu = None
        if world == 1 and not a.no_cpu_baseline:
            cpu = cpu_baseline(a.cpu_mib, a.block_id)
        line = {
            "metric": "device-resident LZ4 GiB/s (compress, decompress) on 4 MiB blocks at 1/2/4/8 MI355X",
            "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": K, "warmup": a.warmup,
            "ms_per_step": round((tc + td) / K * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic (SURVEY.md App. F generator, seed 42)",
            "config": {"workload": (f"configs[2]: {a.gib:g} GiB/GPU pre-compressed synthetic stream, "
                                    f"{bm >> 10} KiB blocks, decompress+XXH32 verify only, device-resident")
                                   if a.decompress_only else
                                   (f"configs[1]: {a.gib:g} GiB/GPU synthetic, {bm >> 10} KiB independent blocks, "
                                    "-Sx -BX frame, compress+decompress+XXH32, device-resident"),
                       "bytes_per_gpu": n, "block_bytes": bm, "parallelism": f"block-sharded x{world}"
                                                                                + (", RCCL gather overlapped with decompress" if world > 1 else "")},
            "compress_GiBps": round(comp_gibps, 3) if comp_gibps else None,
            "decompress_GiBps": round(decomp_gibps, 3),
            "ratio": round(n / frame_len, 4), "frame_bytes": frame_len,
            "stitched_frame_bytes": stitched["len"] if world > 1 else frame_len, "roundtrip_ok": ok,
            "roofline": roof, "decode_roofline": dec_roof, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
