"""bench.py — device-resident LZ4 frame compress + decompress on MI355X.

Workload (BASELINE.json configs[1]): 8 GiB synthetic buffer per GPU
(SURVEY.md App. F generator), 4 MiB independent blocks, -Sx -BX frames
(block XXH32 on, serial content checksum off), compress + decompress +
XXH32, inputs resident in HBM when the timed region starts.

One step at N = 1: compress the buffer into one lz4mt frame, then decompress
that frame (block checksums verified by the decoder).

One step at N > 1 (one process per GPU, RCCL): each
rank owns a contiguous block range (its 8 GiB shard of the 8N GiB stream,
weak scaling).
  compress   = local encode + the RCCL gather of every shard's records into
               ONE frame on rank 0 ("from the first launch to the completed
               gather on the root"); ``gather_ms`` reports the gather alone;
  scatter    = rank 0 walks that frame on the device and sends each rank its
               run of whole records (lz4mt_amd.dist.scatter_frame); timed and
               reported as ``scatter_ms``, outside ``value`` (it moves
               compressed bytes root -> peers; the decompress figure is the
               decoder's);
  decompress = every rank decodes the piece it received.
After the timed steps rank 0 decodes the stitched frame once (untimed) and
compares every shard's chunk digests with the ranks' own (exit 1 on a
mismatch); each rank also compares its decoded piece with its source.

Prints ONE JSON line on rank 0: value = uncompressed GiB of the whole job /
(compress + decompress time), the per-direction rates, the encode kernel's
roofline (HIP events on the library's launch stream; HBM traffic from the
committed PMC profile of this same configuration, calibrated) and the CPU
baseline (lz4mt-shaped pipeline on the host cores over liblz4 when present).
"""
import argparse
import contextlib
import ctypes
import json
import os
import socket
import subprocess
import sys
import tempfile
import threading
import time
import traceback

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# torch, torch.distributed and lz4mt_amd (which loads the HIP library) are
# imported in main(): with --gpus N > 1 and no WORLD_SIZE, the parent only
# launches the N ranks and must not touch the GPU first.
torch = dist = L = D = None

GiB = float(1 << 30)
METRIC = "device-resident LZ4 GiB/s (compress, decompress) on 4 MiB blocks at 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
GOLDEN = 0x9E3779B97F4A7C15
# the headline's PMC profile; the sweep points' are profiles/pmc_b<id>.json
PMC_PROFILE = os.path.join(ROOT, "profiles", "pmc_current.json")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--gib", type=float, default=8.0, help="GiB per GPU (weak scaling, the default)")
    p.add_argument("--total-gib", type=float, default=None,
                   help="strong scaling: ONE buffer of this many GiB, block-sharded over the ranks "
                        "(configs[3]: --total-gib 64 at 1/2/4/8 GPUs)")
    p.add_argument("--block-id", type=int, default=7, help="4..7 = 64 KiB..4 MiB")
    p.add_argument("--stream-checksum", action="store_true",
                   help="default lz4mt flags (FLG.2 content checksum, no block checksum) instead of -Sx -BX")
    p.add_argument("--level", type=int, default=0, help="compression level: 3..9 = LZ4-HC (not the headline)")
    p.add_argument("--block-dependent", action="store_true", help="-BD frames (serial; not the headline)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-mib", type=int, default=1024, help="CPU baseline sample (MiB, all threads)")
    p.add_argument("--gather", choices=["streamed", "after"], default="streamed",
                   help="N > 1: stream the shards' records to rank 0 while they encode (dist.compress_gather_streamed), "
                        "or gather each finished shard frame after its encode (dist.gather_frame)")
    p.add_argument("--transport", choices=["ipc", "rccl"], default="ipc",
                   help="streamed gather: packs pushed by copy engines into IPC-shared root buffers (default; RCCL "
                        "kernels need LDS that the running encodes hold), or RCCL point-to-point")
    p.add_argument("--decompress-only", action="store_true",
                   help="configs[2]: time only the decompression of a pre-compressed stream (use --gib 32)")
    return p.parse_args()


def timings():
    ms = (ctypes.c_float * 4)()
    if L.lib.lz4mtHipGetTimings(ms) != 0:
        return None
    return list(ms)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def usable_cores():
    """Threads for the reference's pool here: hardware_concurrency()
    (src/lz4mt_compat.cpp, nPool = hw + 1, src/lz4mt.cpp:281), bounded by
    what this process may actually run on -- its CPU affinity, its cgroup
    CPU quota and the box's per-job thread share (OMP_NUM_THREADS /
    MAX_JOBS, set by the GPU pool to the lease's CPU share).  Threads beyond
    that only contend.  Returns (threads, hardware_concurrency, limits) with
    every limit seen and the one that set the count."""
    hw = os.cpu_count() or 1
    lim = {"hardware_concurrency": hw}
    if hasattr(os, "sched_getaffinity"):
        lim["affinity"] = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        lim["cgroup_quota"] = None if q == "max" else max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    for var in ("OMP_NUM_THREADS", "MAX_JOBS"):
        v = os.environ.get(var, "")
        if v.isdigit() and int(v) > 0:
            lim[var] = int(v)
    cands = {k: v for k, v in lim.items() if isinstance(v, int)}
    by = min(cands, key=lambda k: (cands[k], k != "hardware_concurrency"))
    lim["limited_by"] = by
    return max(1, cands[by]), hw, lim


def cpu_baseline(mib, block_id, sck, level=0, bd=False):
    """The reference's CPU path for this run's codec, timed on the host.

    Independent blocks: the lz4mt-shaped pipeline (one task per block, nPool =
    threads + 1, in-order writer, block/stream XXH32) over the codec lz4mt
    links -- liblz4's LZ4_compress_limitedOutput, or for level >= 3
    LZ4_compressHC2_limitedOutput at that level (src/main.cpp:749-785) --
    when the box has liblz4, else over the oracle's restatements; best of 3
    at full width, one pass single-threaded.  -BD: single-threaded, as
    compressBlockDependency is (src/lz4mt.cpp:460-538, 737-845), one LZ4
    stream over liblz4 (orc_bd_roundtrip).  Rank 0, N = 1, bounded sample."""
    import oracle
    threads, hw, limits = usable_cores()
    n = mib << 20
    buf = ctypes.create_string_buffer(n)
    oracle.lib.orc_gen_synthetic(buf, n, 42)
    p = oracle.params(block_id, stream_checksum=sck, block_checksum=not sck)
    lz = oracle.liblz4_codec()
    flags = ("default flags" if sck else "-Sx -BX") + (f" level {level}" if level >= 3 else "") + (" -BD" if bd else "")
    line = {"unit": "GiB/s", "kind": "port", "hardware_concurrency": hw, "cpu_model": _cpu_model(),
            "thread_limits": limits}
    if bd:
        if not lz:
            return None   # the stream API comes from liblz4 only
        if level >= 3:
            mib = min(mib, 64)   # ~30 MB/s: a bounded sample
        tc, td, _ = oracle.bd_roundtrip(buf, mib << 20, block_id, sck, not sck, lz[2], hc=level >= 3)
        n = mib << 20
        how = ("one HC stream at level 9 (LZ4_compress_HC_continue" if level >= 3 else
               "one LZ4 stream (LZ4_compress_fast_continue")
        line.update({"value": round(n / GiB / (tc + td), 3), "cores": 1, "codec": f"liblz4 {lz[1]}",
                     "sample": f"{mib} MiB App.F synthetic, B{block_id} {flags}: {how}, cap n-1; "
                               f"LZ4_decompress_safe_usingDict), block/stream "
                               f"XXH32, single thread as the reference's -BD path",
                     "compress_GiBps": round(n / GiB / tc, 3), "decompress_GiBps": round(n / GiB / td, 3)})
        return line
    if level >= 3:
        codec = oracle.hc_codec(level, lz[2] if lz else None)
        codec_name = f"liblz4 {lz[1]} HC" if lz else "oracle HC restatement"
    else:
        codec, codec_name = (lz[0], f"liblz4 {lz[1]}") if lz else (None, "oracle restatement")
    n1 = min(n, 256 << 20 if level < 3 else 64 << 20)
    tc1, td1, _ = oracle.pipeline_roundtrip(buf, n1, p, 1, codec)
    # configs[0] as BASELINE.json states it: 256 MiB, 4 MiB blocks, one
    # thread, XXH32 on -- the reference's default flags (content checksum)
    d1 = None
    if level < 3 and not sck:
        pd = oracle.params(block_id, stream_checksum=True, block_checksum=False)
        d1 = oracle.pipeline_roundtrip(buf, n1, pd, 1, codec)[:2]
    best = None
    for _ in range(3 if level < 3 else 1):
        tc, td, _ = oracle.pipeline_roundtrip(buf, n, p, threads, codec)
        if best is None or tc + td < best[0] + best[1]:
            best = (tc, td)
    tcN, tdN = best
    line.update({
        "value": round(n / GiB / (tcN + tdN), 3), "cores": threads, "codec": codec_name,
        "sample": f"{mib} MiB App.F synthetic, B{block_id} {flags}, compress+decompress "
                  f"through an lz4mt-shaped pipeline (nPool=threads+1, in-order writer, checksums) over {codec_name}; "
                  f"best of {3 if level < 3 else 1}; single thread on {n1 >> 20} MiB",
        "compress_GiBps": round(n / GiB / tcN, 3), "decompress_GiBps": round(n / GiB / tdN, 3),
        "single_thread_compress_GiBps": round(n1 / GiB / tc1, 3),
        "single_thread_decompress_GiBps": round(n1 / GiB / td1, 3)})
    if d1:
        line["configs0_single_thread_default_flags"] = {
            "sample": f"{n1 >> 20} MiB App.F, B{block_id}, default flags (FLG.2 content XXH32), one thread",
            "compress_GiBps": round(n1 / GiB / d1[0], 3), "decompress_GiBps": round(n1 / GiB / d1[1], 3)}
    return line


def pmc_traffic(kernel, n, bm, flg):
    """HBM bytes per launch of ``kernel`` from profiles/pmc_current.json, which
    tools/prof.sh + tools/pmcsum.py write for one named configuration; used
    only when that configuration is this run's (else None + the reason).
    FETCH_SIZE is divided by the calibration the profile measured on a known
    byte count (MI355X_MICROARCH.md: gfx950 FETCH_SIZE is ~1/2 of wide
    streaming reads; other widths need their own calibration)."""
    import glob
    prof, seen, used = None, [], None
    for path in [PMC_PROFILE] + sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_b*.json"))
                                       + glob.glob(os.path.join(ROOT, "profiles", "pmc_dec*.json"))):
        try:
            p = json.load(open(path))
        except (OSError, ValueError):
            continue
        cfg = p.get("config", {})
        seen.append(cfg.get("workload", os.path.basename(path)))
        if (cfg.get("bytes"), cfg.get("block_bytes"), cfg.get("flg")) == (n, bm, flg):
            prof, used = p, os.path.relpath(path, ROOT)
            break
    if prof is None:
        return None, f"no PMC profile of this configuration (have: {seen})"
    k = prof.get("kernels", {}).get(kernel)
    if not k:
        return None, f"{kernel} not in the profile"
    cal = prof.get("calibration", {}).get(kernel) or {}
    fr = k["fetch_bytes"]
    if "stream_factor" in cal:   # a streamed part of known size + the rest at its own factor
        sb = cal["stream_bytes"]
        fetch = sb + max(0.0, fr - cal["stream_factor"] * sb) / cal["other_factor"]
    else:
        fetch = fr / cal.get("fetch_factor", 0.5)
    return {"bytes": fetch + k["write_bytes"], "raw_bytes": fr + k["write_bytes"], "fetch_raw": fr,
            "fetch_calibrated": round(fetch),
            "write": k["write_bytes"], "calibration": cal.get("how", "guide x2 (uncalibrated)"),
            "source": f"{used} ({prof.get('tag', '?')})"}, None


@contextlib.contextmanager
def stdout_to_stderr():
    """gloo prints '[Gloo] Rank r is connected to k peer ranks' on file
    descriptor 1 when a group connects (the gloo control group of every N > 1
    run too); the driver reads stdout for rank 0's one JSON line, so group
    set-up writes to stderr instead."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def frame_encoder(bm):
    """The kernel lz4mtHipCompressFrameAsyncEx runs for bm-byte blocks
    (launch_encode, lz4mt_kernels.hip): the byU16 table below 65 547 B, the
    3-byte table at 256 KiB (LZ4MT_AMD_ENC overrides), else k_encode."""
    enc = os.environ.get("LZ4MT_AMD_ENC", "")
    if bm < 65547:
        return "k_encode16"
    if enc == "p17" or (enc != "base" and bm <= (256 << 10)):
        return "k_encode_p17"
    return "k_encode"


class RunGuard:
    """Bounded, diagnosable N > 1 runs.

    Every rank names the stage it is in (init, input, setup, step, check,
    report).  Whatever ends a rank early -- an exception in any stage, or
    the run passing its deadline (LZ4MT_BENCH_DEADLINE_S, default 300 s from
    the moment torch is imported; a collective that never returns counts) --
    ends the WHOLE run the same way: rank 0 prints ONE JSON line
    (``status: "failed"``, the failing ``stage``, ``transport``, ``error``,
    and every rank's report in ``failures``) and exits non-zero.
      * a non-root rank writes its report into a per-run directory (all
        ranks of one node share it: /tmp keyed by the rendezvous port and
        the launcher's pid) and waits up to 20 s for rank 0 to acknowledge;
      * rank 0 polls that directory from a thread, so it reports even while
        its main thread is blocked inside a collective that waits for the
        failed rank; on its own exception it first waits ~2 s for the other
        ranks' reports (its error may be the echo of theirs, e.g. a gloo
        connection closed by a dead peer);
      * the earliest report is the cause (``stage``/``error``).
    Processes end with os._exit, so no process-group destructor can stall
    the exit.  The process groups' timeout is set above the deadline
    (bench.py), so the guard, not a watchdog abort, ends a hung collective.
    LZ4MT_BENCH_FAULT="<stage>:<rank>[:hang]" injects a failure (or a hang)
    at a stage on one rank, for the tests."""

    STAGES = ("init", "input", "setup", "step", "check", "report")

    def __init__(self, rank, world, n_gpus, enabled, deadline_s=None):
        self.rank, self.world, self.n_gpus, self.enabled = rank, world, n_gpus, enabled
        self.stage, self.transport = "init", None
        self.deadline_s = float(deadline_s if deadline_s is not None else
                                os.environ.get("LZ4MT_BENCH_DEADLINE_S", "300"))
        self.t0 = time.monotonic()
        self._lock = threading.Lock()
        self._reported = False
        # the line goes to the process's real stdout even while a group set-up
        # has file descriptor 1 redirected to stderr (stdout_to_stderr)
        self._out_fd = os.dup(1)
        key = f"{os.environ.get('MASTER_PORT', '0')}_{os.getppid()}"
        self.dir = os.path.join(tempfile.gettempdir(), f"lz4mt_bench_{key}")
        f = os.environ.get("LZ4MT_BENCH_FAULT", "").split(":")
        self.fault = (f[0], int(f[1]) if len(f) > 1 and f[1].isdigit() else 0, len(f) > 2 and f[2] == "hang") \
            if f[0] else None
        if enabled:
            os.makedirs(self.dir, exist_ok=True)
            threading.Thread(target=self._deadline, daemon=True).start()
            if rank == 0 and world > 1:
                threading.Thread(target=self._poll, daemon=True).start()

    def remaining_s(self):
        return self.deadline_s - (time.monotonic() - self.t0)

    def enter(self, stage, point=None):
        """Now in ``stage``; ``point`` names a place inside it (a fault can
        be injected there: e.g. "gather", between a step's gather and its
        scatter, while the other ranks sit in a collective)."""
        self.stage = stage
        if self.fault and self.fault[0] == (point or stage) and self.fault[1] == self.rank:
            if self.fault[2]:
                print(f"bench.py: rank {self.rank}: injected hang in stage {stage}", file=sys.stderr, flush=True)
                while True:
                    time.sleep(3600)
            raise RuntimeError(f"injected fault (LZ4MT_BENCH_FAULT) in stage {stage} on rank {self.rank}")

    def _record(self, error):
        return {"rank": self.rank, "stage": self.stage, "transport": self.transport, "error": error,
                "t": time.time(), "elapsed_s": round(time.monotonic() - self.t0, 3)}

    def _reports(self):
        out = []
        try:
            names = sorted(os.listdir(self.dir))
        except OSError:
            return out
        for nm in names:
            if nm.startswith("fail_") and nm.endswith(".json"):
                try:
                    out.append(json.load(open(os.path.join(self.dir, nm))))
                except (OSError, ValueError):
                    pass
        return out

    def failed(self, error):
        """This rank cannot go on: report (rank 0: the JSON line) and exit 1."""
        rec = self._record(error)
        print(f"bench.py: rank {self.rank} failed in stage {self.stage}: {error}", file=sys.stderr, flush=True)
        if self.rank == 0:
            time.sleep(2.0)   # the other ranks' reports, if this error echoes theirs
            self._report_root([rec] + self._reports())
        else:
            try:
                os.makedirs(self.dir, exist_ok=True)
                tmp = os.path.join(self.dir, f".fail_{self.rank}.tmp")
                with open(tmp, "w") as fh:
                    json.dump(rec, fh)
                os.replace(tmp, os.path.join(self.dir, f"fail_{self.rank}.json"))
            except OSError:
                pass
            ack = os.path.join(self.dir, "ack")
            t_end = time.monotonic() + 20.0
            while time.monotonic() < t_end and not os.path.exists(ack):
                time.sleep(0.1)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(1)

    def _report_root(self, recs):
        with self._lock:
            if self._reported:
                return
            self._reported = True
        recs = sorted(recs, key=lambda r: r.get("t", 0.0))
        first = recs[0]
        line = {"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": self.n_gpus, "status": "failed",
                "stage": first.get("stage"), "transport": first.get("transport") or self.transport,
                "error": first.get("error"), "failed_rank": first.get("rank"), "root_stage": self.stage,
                "elapsed_s": round(time.monotonic() - self.t0, 3), "deadline_s": self.deadline_s,
                "failures": [{k: r.get(k) for k in ("rank", "stage", "transport", "error", "elapsed_s")}
                             for r in recs]}
        sys.stdout.flush()
        os.write(self._out_fd, (json.dumps(line) + "\n").encode())
        try:
            open(os.path.join(self.dir, "ack"), "w").close()
        except OSError:
            pass

    def _poll(self):
        while True:
            time.sleep(0.2)
            with self._lock:
                if self._reported:
                    return
            recs = self._reports()
            if recs:
                time.sleep(1.0)   # the rest of a cascade
                self._report_root(self._reports() + [self._record("(rank 0 was still running this stage)")])
                sys.stdout.flush()
                sys.stderr.flush()
                os._exit(1)

    def _deadline(self):
        while self.remaining_s() > 0:
            time.sleep(min(1.0, max(0.05, self.remaining_s())))
        with self._lock:
            done = self._reported
        if done:   # the result is out; only the teardown (process-group destroy) is late
            print("bench.py: teardown passed the deadline; exiting", file=sys.stderr, flush=True)
            sys.stdout.flush()
            os._exit(self._exit_code)
        self.failed(f"deadline exceeded: the run passed LZ4MT_BENCH_DEADLINE_S = {self.deadline_s:g} s "
                    f"in stage {self.stage} (a collective or a peer that never answered)")

    _exit_code = 0

    def succeeded(self, ok=True):
        """The run's result is final on this rank; rank 0 prints its line only
        when this returns True (under the same lock as a failure line: never
        two lines).  The deadline still bounds the teardown after it."""
        with self._lock:
            if self._reported:
                return False
            self._reported = True
            self._exit_code = 0 if ok else 1
        return True

    def cleanup(self):
        if self.enabled and self.rank == 0:
            import shutil
            shutil.rmtree(self.dir, ignore_errors=True)


def workload_id(world, block_id, sck=False, level=0, bd=False, n_total=None, strong=False):
    """configs[1] is the 4 MiB -Sx -BX headline; other block sizes are the
    configs[4] sweep.  N > 1 is labelled configs[3] only when the run IS
    configs[3] -- 64 GiB in total of 4 MiB -Sx -BX blocks (weak scaling at
    8 GPUs x 8 GiB, or --total-gib 64 at any N); any other N > 1 run says
    what it is.  The content checksum (default flags),
    LZ4-HC levels and -BD are modes BASELINE.json names no config for:
    labelled as such, never as configs[1]."""
    if sck or level >= 3 or bd:
        mode = ", ".join(m for m, on in (("default flags (FLG.2 content checksum)", sck),
                                         (f"LZ4-HC level {level}", level >= 3), ("-BD", bd)) if on)
        return f"off-baseline mode ({mode}; not a BASELINE.json config)"
    if world > 1 or strong:
        shape = (f"strong scaling, one {n_total / GiB:g} GiB buffer over {world} GPU(s)" if strong else
                 f"weak scaling, {n_total / world / GiB:g} GiB/GPU x {world} = {n_total / GiB:g} GiB")
        if n_total == 64 * (1 << 30) and block_id == 7:
            return f"configs[3] ({shape})"
        return f"configs[3]-style scaling point, not configs[3] itself ({shape}; configs[3] is 64 GiB in total)"
    return "configs[1]" if block_id == 7 else "configs[4] (block-size sweep)"


def parallelism_label(world, distributed, streamed, transport_name, backend):
    """What actually moved the records (no 'RCCL gather'
    when the IPC push did it)."""
    s = f"block-sharded x{world}"
    if not distributed:
        return s
    if streamed:
        how = ("copy-engine IPC push into the root's receive buffers, round sizes over gloo"
               if transport_name == "ipc" else
               f"{'RCCL' if backend == 'nccl' else backend} point-to-point ({transport_name})")
        return s + f", records gathered to one frame on rank 0 beside the encodes by {how}"
    return s + f", records gathered to one frame on rank 0 after the encode by " \
               f"{'RCCL' if backend == 'nccl' else backend} point-to-point"


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(a):
    """--gpus N > 1 without a torch.distributed launcher: start one rank per
    GPU as a CHILD process (python -m torch.distributed.run, rendezvous on
    127.0.0.1) and exit with its status.  Nothing here has touched the GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    global torch, dist, L, D
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world} ranks were launched")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch as _torch
    import torch.distributed as _dist
    torch, dist = _torch, _dist
    # LZ4MT_BENCH_DIST=1 runs the N > 1 path (process group, streamed gather,
    # scatter, stitched-frame check) at world size 1 too: the nccl backend on
    # a one-GPU box (RCCL allows one rank per device)
    distributed = world > 1 or os.environ.get("LZ4MT_BENCH_DIST") == "1"
    guard = RunGuard(rank, world, a.gpus, enabled=distributed)
    try:
        run(a, guard, world, rank, local, distributed)
    except BaseException as e:   # noqa: B902 -- every way out of a rank ends the run the same way
        if not guard.enabled or (isinstance(e, SystemExit) and (e.code in (0, None) or guard._reported)):
            raise   # (a result line is out already: its exit status stands)
        err = f"{type(e).__name__}: {e}"
        traceback.print_exc(file=sys.stderr)
        guard.failed(err)


def run(a, guard, world, rank, local, distributed):
    global L, D
    import lz4mt_amd as _L
    from lz4mt_amd import dist as _D
    L, D = _L, _D
    # LZ4MT_BENCH_BACKEND=gloo rehearses the N > 1 orchestration with several
    # ranks sharing the GPUs there are (gloo moves CUDA tensors through the
    # host); the measured multi-GPU path is RCCL, one rank per GPU
    backend = os.environ.get("LZ4MT_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count()) if backend != "nccl" else local
    torch.cuda.set_device(local)
    if distributed:
        guard.enter("init")
        # an explicit timeout: a rank that stops answering ends the run
        # non-zero instead of stalling it for torch's 30 min default; set
        # above the guard's deadline, so the guard (one JSON line) and not
        # the RCCL watchdog's abort ends a collective that never returns
        import datetime
        pg_timeout = max(D.dist_timeout(), datetime.timedelta(seconds=guard.deadline_s + 60))
        with stdout_to_stderr():
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=pg_timeout)
            else:
                dist.init_process_group(backend, timeout=pg_timeout)
                dist.barrier()   # (gloo connects its mesh here at the latest)
        guard.enter("input")
    dev = torch.device("cuda", local)
    stream = torch.cuda.current_stream()

    bm = 1 << (8 + 2 * a.block_id)
    if a.total_gib is not None:   # strong scaling: rank r owns shard_blocks' range of ONE buffer
        n_total = int(a.total_gib * GiB) // bm * bm
        first_byte, n, _, _ = D.shard_blocks(n_total, bm, world, rank)
    else:                         # weak scaling: --gib per rank, rank r = shard r of one global stream
        n = int(a.gib * GiB) // bm * bm
        first_byte, n_total = rank * n, n * world
    seed = (42 + (first_byte // 65536) * GOLDEN) % (1 << 64)   # App. F segment index of the shard's start
    src = L.gen_synthetic(n, seed=seed, device=dev)
    sck = a.stream_checksum
    if sck and distributed:
        raise SystemExit("the content checksum (FLG.2) is one serial chain over the whole stream: it does not shard")
    sd = L.make_sd(a.block_id, stream_checksum=sck, block_checksum=not sck, block_dependence=a.block_dependent)
    flg = (0x64 if sck else 0x70) & ~(0x20 if a.block_dependent else 0)
    if (a.level >= 3 or a.block_dependent) and distributed:
        raise SystemExit("--level / --block-dependent are single-GPU measurements")
    streamed = distributed and a.gather == "streamed" and not a.decompress_only
    cap = L.frame_bound(n, sd)
    # the streamed gather builds the frame on rank 0 from the shard workspace:
    # no per-rank frame buffer or frame workspace (8 + 8 GiB per GPU spared)
    frame_buf = None if streamed else torch.empty(cap, dtype=torch.uint8, device=dev)
    ws = None if streamed else L.compress_workspace(n, sd, device=dev, level=a.level)
    out = torch.empty(n + (1 << 20), dtype=torch.uint8, device=dev)
    fsz = torch.zeros(2, dtype=torch.int64, device=dev)

    def compress():
        if sck:   # the synchronous call: the serial content checksum runs on the host beside the encode
            hs = ctypes.c_uint64(0)
            r = L.lib.lz4mtHipCompressFrameEx(
                ctypes.c_void_p(src.data_ptr()), n, ctypes.c_void_p(frame_buf.data_ptr()), cap, ctypes.byref(hs),
                ctypes.byref(sd), a.level, ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                ctypes.c_void_p(stream.cuda_stream))
            fsz[0] = hs.value
        else:
            r = L.lib.lz4mtHipCompressFrameAsyncEx(
                ctypes.c_void_p(src.data_ptr()), n, ctypes.c_void_p(frame_buf.data_ptr()), cap,
                ctypes.c_void_p(fsz.data_ptr()), ctypes.byref(sd), a.level, ctypes.c_void_p(ws.data_ptr()),
                ws.numel(), ctypes.c_void_p(stream.cuda_stream))
        if r != 0:
            raise L.Lz4MtError(r, "compress")

    def decompress(fr, flen):
        osz = ctypes.c_uint64(0)
        sdo = L.init_stream_descriptor()
        r = L.lib.lz4mtHipDecompressFrame(ctypes.c_void_p(fr.data_ptr()), flen,
                                          ctypes.c_void_p(out.data_ptr()), out.numel(), ctypes.byref(osz),
                                          ctypes.byref(sdo), ctypes.c_void_p(stream.cuda_stream))
        if r != 0 or osz.value != n:
            raise L.Lz4MtError(r, f"decompress ({osz.value} of {n} bytes)")

    def sync_all():
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        return time.perf_counter()

    if a.decompress_only:   # compress once, untimed
        compress()
        torch.cuda.synchronize()
    own_body = 0
    transport = transport_name = None
    if distributed:
        guard.transport = (a.transport if streamed else f"{backend} point-to-point (gather after the encode)")
        guard.enter("setup")
    if streamed:   # the shard engine's streams and workspace, the control group and transport, made once
        eng = D.HipShardEngine(dev)
        shard_ws = L.shard_workspace(n, sd, device=dev)
        with stdout_to_stderr():
            ctrl = D.control_group()
            dist.barrier(group=ctrl)   # (connected inside the redirect)
        transport = D.IpcPushTransport(dev) if a.transport == "ipc" else D.RcclTransport()
        transport_name = a.transport
        peers = D.peer_access_matrix() if rank == 0 else None
        # the transport's set-up (IPC buffers, maps, the pattern check) before
        # any step: collective, and on failure every rank falls back together
        try:
            D.prepare_transport(transport, eng, n, sd, ctrl=ctrl)
        except D.IpcSetupError as e:
            print(f"bench.py: IPC PUSH UNAVAILABLE ({e}); streamed gather falls back to RCCL point-to-point",
                  file=sys.stderr, flush=True)
            transport, transport_name = D.RcclTransport(), f"rccl (IPC setup failed: {e})"
            guard.transport = transport_name
            D.prepare_transport(transport, eng, n, sd, ctrl=ctrl)
    if distributed:
        guard.enter("step")

    def run_steps(transport):
        """W untimed + K timed steps; returns the accumulated timings and the last step's frames."""
        R = dict(tc=0.0, td=0.0, ts=0.0, tg=0.0, enc_ms=[], dec_ms=[], frame_len=0, exposed_ms=[], rounds=[],
                 tails=[], scat=[], full=None, piece=None, own_body=0)
        L.lib.lz4mtHipSetTiming(1)
        for it in range(a.warmup + a.steps):
            timed = it >= a.warmup
            t0 = sync_all()
            tm = None
            tgr = 0.0
            if streamed:   # encode + streamed gather: ONE frame on rank 0
                st_ = {}
                R["full"] = D.compress_gather_streamed(src, sd, dst=0, engine=eng, ws=shard_ws, stats=st_,
                                                       transport=transport, ctrl=ctrl)
                end_ev = torch.cuda.Event(enable_timing=True)
                end_ev.record()
                torch.cuda.synchronize()
                t1 = sync_all()
                tm = [eng.enc_start.elapsed_time(eng.enc_done)]
                R["exposed_ms"].append(eng.enc_done.elapsed_time(end_ev) if rank == 0 else 0.0)
                tgr = R["exposed_ms"][-1] * 1e-3
                R["rounds"].append(st_.get("rounds", 0))
                R["tails"].append((st_.get("tail_rounds_s") or 0.0, st_.get("rounds_after_encode", 0)))
                R["frame_len"] = R["full"].numel() if rank == 0 else 0
                R["own_body"] = st_.get("own_body_bytes", 0)
            else:
                if not a.decompress_only:
                    compress()
                R["frame_len"] = int(fsz[0].item())          # synchronises the stream
                if not a.decompress_only:
                    tm = timings()
                tl = time.perf_counter()
                if distributed:   # the gather belongs to compress
                    R["full"] = D.gather_frame(frame_buf, R["frame_len"], dst=0)
                    torch.cuda.synchronize()
                t1 = sync_all()
                tgr = time.perf_counter() - tl if distributed else 0.0
            full = R["full"]
            if distributed:
                guard.enter("step", point="gather")
                sst = {}
                R["piece"] = D.scatter_frame(full if rank == 0 else None, full.numel() if rank == 0 else 0, src=0,
                                             device=dev, stats=sst)
                if timed:
                    R["scat"].append(sst)
                torch.cuda.synchronize()
                t2 = sync_all()
            else:
                R["piece"], t2 = frame_buf, t1
            piece = R["piece"]
            decompress(piece, piece.numel() if distributed else R["frame_len"])
            tmd = timings()
            t3 = sync_all()
            if timed:
                R["tc"] += t1 - t0
                R["ts"] += t2 - t1
                R["td"] += t3 - t2
                R["tg"] += tgr
                if tm:
                    R["enc_ms"].append(tm[0])
                if tmd:
                    R["dec_ms"].append(tmd[1])
        L.lib.lz4mtHipSetTiming(0)
        return R

    def check(R):
        """Correctness (not timed): this rank's decoded piece == its source; at
        N > 1 the root decodes the stitched frame and checks every shard.
        Returns (this rank's ok, stitched ok (same on every rank) or None)."""
        ok = bool(torch.equal(out[:n], src))
        if not distributed:
            return ok, None

        def digests(t):
            return L.xxh32_chunks(t, 16 << 20).to(torch.int64)

        def decode_full(f):
            o, r = L.decompress_frame(f)
            return o if r == 0 else o[:0]
        return ok, D.verify_stitched(R["full"] if rank == 0 else None, src, decode_full, digests)

    R = run_steps(transport)
    mem = None
    if distributed:
        guard.enter("check")
        # the root's device memory at its peak: torch's allocator (sources,
        # workspaces, mirrors, the stitched frame, pieces) and the device as
        # a whole (hipMemGetInfo: + the IPC receive buffers, library scratch)
        free_b, total_b = torch.cuda.mem_get_info(dev)
        mem = {"max_allocated_GiB": round(torch.cuda.max_memory_allocated(dev) / GiB, 2),
               "device_used_GiB": round((total_b - free_b) / GiB, 2), "device_total_GiB": round(total_b / GiB, 2)}
    ok, stitched_ok = check(R)
    if streamed and stitched_ok is False and isinstance(transport, D.IpcPushTransport):
        # the IPC push delivered a wrong frame although its set-up check
        # passed: measure again over RCCL (every rank sees the same verdict)
        # and say so in the line -- the first measurement is discarded
        print("bench.py: THE STITCHED FRAME OVER THE IPC PUSH FAILED ITS CHECK; steps re-run over RCCL point-to-point",
              file=sys.stderr, flush=True)
        transport.close()
        transport, transport_name = D.RcclTransport(), "rccl (IPC push gave a wrong stitched frame; re-run)"
        guard.transport = transport_name
        guard.enter("setup")
        D.prepare_transport(transport, eng, n, sd, ctrl=ctrl)
        guard.enter("step")
        R = run_steps(transport)
        guard.enter("check")
        ok, stitched_ok = check(R)
    tc, td, ts, tg = R["tc"], R["td"], R["ts"], R["tg"]
    enc_ms, dec_ms, frame_len, exposed_ms = R["enc_ms"], R["dec_ms"], R["frame_len"], R["exposed_ms"]
    rounds, tails, scat, full, own_body = R["rounds"], R["tails"], R["scat"], R["full"], R["own_body"]
    if distributed:
        mem["after_verify_max_allocated_GiB"] = round(torch.cuda.max_memory_allocated(dev) / GiB, 2)
        t = torch.tensor([tc, td, ts, tg, 0.0 if ok else 1.0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        tc, td, ts, tg, bad = t.tolist()
        ok = bad == 0.0 and stitched_ok
        guard.enter("report")
    K = a.steps
    total = n_total * K
    comp_gibps = None if a.decompress_only else total / GiB / tc
    decomp_gibps = total / GiB / td
    value = decomp_gibps if a.decompress_only else total / GiB / (tc + td)

    enc_avg = sum(enc_ms) / len(enc_ms) if enc_ms else None
    dec_avg = sum(dec_ms) / len(dec_ms) if dec_ms else None
    # algorithmic bytes per launch: in + out of this rank's encode
    body = own_body if streamed else frame_len - 7 - 4 - (4 if sck else 0)
    alg = n + body
    # the kernels the timing marks bracket in this mode
    enc_k = ("k_encode_hc_bd" if a.block_dependent and a.level >= 3 else "k_encode_linked_round"
             if a.block_dependent else "k_encode_hc" if a.level >= 3 else
             "k_encode_pub (+ k_xxh32_stored)" if streamed else frame_encoder(bm))
    dec_k = "k_decode_linked" if a.block_dependent else "k_decode"
    roof = dec_roof = None
    if enc_avg:
        ach = alg / (enc_avg * 1e-3) / 1e9
        tr, why = pmc_traffic(enc_k, n, bm, flg)
        roof = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBPS, 5), "traffic": round(tr["bytes"]) if tr else None,
                "kernel": enc_k + (" (+ k_hc_prev_seg)" if a.block_dependent and a.level >= 3 else
                                   " (+ k_link_settle rounds, serial fallback)" if a.block_dependent else
                                   " (+ k_hc_prev)" if a.level >= 3 else ""),
                "kernel_ms": round(enc_avg, 3), "algorithmic_bytes": alg,
                "traffic_detail": tr or why}
    if dec_avg:
        ach = alg / (dec_avg * 1e-3) / 1e9
        tr, why = pmc_traffic(dec_k, n, bm, flg)
        dec_roof = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBPS, 5), "traffic": round(tr["bytes"]) if tr else None,
                    "kernel": dec_k, "kernel_ms": round(dec_avg, 3), "algorithmic_bytes": alg,
                    "traffic_detail": tr or why}
    if a.decompress_only and dec_roof:   # the decode kernel is the dominant one here
        roof = dec_roof
    if rank == 0:
        cpu = None
        if world == 1 and not a.no_cpu_baseline:
            cpu = cpu_baseline(a.cpu_mib if a.level < 3 and not a.block_dependent else min(a.cpu_mib, 256),
                               a.block_id, sck, a.level, a.block_dependent)
        flags = ("default flags (FLG.2 content checksum)" if sck else "-Sx -BX") + \
            (" -BD" if a.block_dependent else "") + (f" level {a.level} (LZ4-HC)" if a.level >= 3 else "")
        line = {
            "metric": "device-resident LZ4 GiB/s (compress, decompress) on 4 MiB blocks at 1/2/4/8 MI355X",
            "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": K, "warmup": a.warmup,
            "ms_per_step": round((tc + td) / K * 1e3, 3), "higher_is_better": True, "scaling": "strong" if a.total_gib is not None else "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic (SURVEY.md App. F generator, seed 42)",
            "config": {"workload": (f"configs[2]: {a.gib:g} GiB/GPU pre-compressed synthetic stream, "
                                    f"{bm >> 10} KiB blocks, decompress+XXH32 verify only, device-resident")
                                   if a.decompress_only else
                                   (f"{workload_id(world, a.block_id, sck, a.level, a.block_dependent, n_total, True)}: "
                                    f"ONE {a.total_gib:g} GiB synthetic buffer block-sharded over "
                                    f"{world} GPU(s), {bm >> 10} KiB independent blocks, {flags} frame, "
                                    f"compress+decompress+XXH32, device-resident")
                                   if a.total_gib is not None else
                                   (f"{workload_id(world, a.block_id, sck, a.level, a.block_dependent, n_total)}: "
                                    f"{a.gib:g} GiB/GPU synthetic, {bm >> 10} KiB "
                                    f"independent blocks, {flags} frame, compress+decompress+XXH32, device-resident"),
                       "bytes_per_gpu": n, "bytes_total": n_total, "block_bytes": bm,
                       "parallelism": parallelism_label(world, distributed, streamed, transport_name, backend)},
            "compress_GiBps": round(comp_gibps, 3) if comp_gibps else None,
            "decompress_GiBps": round(decomp_gibps, 3),
            "ratio": round((n_total / frame_len) if streamed else (n / frame_len), 4), "frame_bytes": frame_len,
            "roundtrip_ok": ok, "roofline": roof, "decode_roofline": dec_roof, "cpu_baseline": cpu,
        }
        if streamed:   # root's GPU time from its own encode's end to the assembled frame
            line.update({"gather": f"streamed beside the encode (dist.compress_gather_streamed, {transport_name})",
                         "ipc_buffers": getattr(transport, "kind", None),
                         "gather_exposed_ms": round(sum(exposed_ms[a.warmup:]) / max(1, K), 3),
                         "gather_rounds": round(sum(rounds[a.warmup:]) / max(1, K), 1),
                         "gather_tail_rounds": round(sum(t[1] for t in tails[a.warmup:]) / max(1, K), 1),
                         "gather_tail_rounds_ms": round(sum(t[0] for t in tails[a.warmup:]) / max(1, K) * 1e3, 3)})
        elif distributed:
            line.update({"gather": "after the encode (dist.gather_frame)"})
        if distributed:
            def avg(k):
                return round(sum(x[k] for x in scat) / max(1, len(scat)) * 1e3, 3)
            line.update({"backend": backend, "transport": transport_name if streamed else backend,
                         "gather_ms": round(tg / K * 1e3, 3), "scatter_ms": round(ts / K * 1e3, 3),
                         "scatter_split_ms": {"walk": avg("walk_s"), "table": avg("table_s"), "p2p": avg("p2p_s"),
                                              "assemble": avg("assemble_s"),
                                              "host_staged": bool(scat and scat[0]["host_staged"])},
                         "root_memory": mem, "peer_access": peers if streamed else D.peer_access_matrix(),
                         "stitched_frame_bytes": full.numel(), "stitched_frame_ok": stitched_ok,
                         "roundtrip_with_scatter_GiBps": round(total / GiB / (tc + ts + td), 3),
                         "deadline_s": guard.deadline_s, "elapsed_s": round(time.monotonic() - guard.t0, 3)})
        if guard.succeeded(ok):
            print(json.dumps(line), flush=True)
    else:
        guard.succeeded(ok)
    if streamed:
        transport.close()
    if distributed:
        dist.destroy_process_group()
    guard.cleanup()
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
