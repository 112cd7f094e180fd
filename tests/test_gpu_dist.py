"""bench.py's multi-GPU entry on a real device.

`python bench.py --gpus N` with no WORLD_SIZE must start N ranks itself
(before anything touches the GPU) and run the block-sharded path of
SURVEY.md §8(e): local encodes, the gather of every shard's records into
ONE frame on rank 0, the device-walk scatter (lz4mtHipFrameRecords) back to
the ranks, and the stitched-frame check over HIP chunk digests
(dist.verify_stitched).  On the one-GPU test box the two ranks share cuda:0
and talk over gloo (LZ4MT_BENCH_BACKEND=gloo; gloo carries the CUDA tensors
through the host) -- the same orchestration the driver's 8-GPU run does over
RCCL.  Reference for the sharding: independent blocks, src/lz4mt.cpp:914-918,
991-995."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _qget(q, procs, timeout):
    """q.get that fails at once when a rank process died without answering
    (instead of waiting out the whole timeout while its peer blocks)."""
    import queue
    import time
    t_end = time.monotonic() + timeout
    while True:
        try:
            return q.get(timeout=2)
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, f"a rank exited with {dead} before answering"
            assert time.monotonic() < t_end, "no answer from the ranks"


def _bench(*args, timeout=300):
    env = dict(os.environ, LZ4MT_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.gpu
def test_bench_gpus2_launches_two_ranks_weak():
    line = _bench("--gpus", "2", "--gib", "0.25", "--steps", "1", "--warmup", "0", "--no-cpu-baseline")
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["stitched_frame_ok"] is True and line["roundtrip_ok"] is True
    assert line["config"]["bytes_total"] == 2 * line["config"]["bytes_per_gpu"]
    # streamed gather (the default): the frame on rank 0 is ONE frame of the
    # whole 2 x 0.25 GiB stream, gathered in rounds beside the encodes
    assert line["gather"].startswith("streamed") and line["gather_rounds"] >= 1
    assert line["stitched_frame_bytes"] == line["frame_bytes"]
    assert 1.9 < line["ratio"] < 2.2
    # the N > 1 line reports what the 8-GPU run needs read:
    # backend, transport, the root's memory, the peer-access matrix and the
    # scatter's parts; gloo moves device pieces through pinned host copies
    assert line["backend"] == "gloo" and line["transport"] == "ipc"
    assert line["root_memory"]["max_allocated_GiB"] > 0 and line["root_memory"]["device_used_GiB"] > 0
    assert line["peer_access"] and all(row[i] for i, row in enumerate(line["peer_access"]))
    sp = line["scatter_split_ms"]
    assert sp["host_staged"] is True and sp["p2p"] >= 0 and sp["walk"] >= 0
    assert line["scatter_ms"] < 5000   # round 3's gloo scatter read device memory through the host: 11.2 s


@pytest.mark.gpu
def test_bench_gpus2_gather_after_encode():
    line = _bench("--gpus", "2", "--gib", "0.25", "--steps", "1", "--warmup", "0", "--no-cpu-baseline",
                  "--gather", "after")
    assert line["n_gpus"] == 2 and line["gather"].startswith("after")
    assert line["stitched_frame_ok"] is True and line["roundtrip_ok"] is True
    # frame_bytes: rank 0's own shard frame; the stitched frame holds both shards' records
    assert line["stitched_frame_bytes"] > line["frame_bytes"]


@pytest.mark.gpu
def test_bench_gpus2_strong_scaling_one_buffer():
    # 0.5 GiB of 4 MiB blocks = 128 blocks, 64 per rank: the two shards are
    # consecutive pieces of ONE App. F buffer, stitched into one frame
    line = _bench("--gpus", "2", "--total-gib", "0.5", "--steps", "1", "--warmup", "0", "--no-cpu-baseline")
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["bytes_total"] == 1 << 29
    assert line["stitched_frame_ok"] is True and line["roundtrip_ok"] is True


def _streamed_rank(rank, world, port, n, bid, cap, kind, q):
    """One rank of a streamed gather on the shared test GPU (gloo): its shard
    of a mixed input (App. F text with incompressible stretches, so some
    blocks are stored raw and their source bytes travel in the last round)."""
    import torch.distributed as dist

    import oracle
    from lz4mt_amd import dist as D
    import lz4mt_amd as L
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def make(n, seed):
            data = bytearray(oracle.gen_synthetic(n, seed))
            rnd = oracle.gen_random(n, seed + 5)
            for s in range(0, n, 5 << 20):
                data[s:s + 1_200_000] = rnd[s:s + 1_200_000]
            return data

        bm = 1 << (8 + 2 * bid)
        sd = L.make_sd(bid, stream_checksum=False, block_checksum=True)
        st = {}
        tr = D.IpcPushTransport(torch.device("cuda", 0)) if kind == "ipc" else D.RcclTransport()
        eng = D.HipShardEngine(torch.device("cuda", 0))
        results = []
        ws = None
        # three calls on one engine and transport: the same layout twice with
        # DIFFERENT inputs into ONE reused workspace (its round state must be
        # reset before the packs read it; the IPC buffers are reused), then a
        # shorter stream (another layout: the IPC buffers are set up again)
        for total, seed in ((n, 42), (n, 7), (n - 3 * bm, 11)):
            data = make(total, seed)
            off, ln, _, _ = D.shard_blocks(total, bm, world, rank)
            src = torch.frombuffer(bytearray(data[off:off + ln]), dtype=torch.uint8).cuda()
            if ws is None or total != n:
                ws = L.shard_workspace(ln, sd)
            full = D.compress_gather_streamed(src, sd, per_block_cap=cap, stats=st, min_round_s=0.0005,
                                              transport=tr, engine=eng, ws=ws)
            if rank == 0:
                want = L.compress_frame(torch.frombuffer(data, dtype=torch.uint8).cuda(), sd)
                results.append(full.numel() == want.numel() and bool(torch.equal(full, want)))
        tr.close()
        if rank == 0:
            q.put((all(results), st["rounds"], results))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["ipc", "rccl"])
@pytest.mark.parametrize("n,bid,cap", [((48 << 20) + 12345, 7, 128 << 10), ((40 << 20) + 7, 6, 16 << 10),
                                       ((12 << 20) + 99, 5, 64 << 10)])
def test_streamed_gather_on_device(n, bid, cap, kind):
    """dist.compress_gather_streamed with the HIP engine, 2 ranks on one GPU:
    k_encode_pub publishes while it encodes (1 and 4 MiB blocks), rounds of
    k_shard_plan / k_shard_pack travel to rank 0 and k_shard_unpack places
    them, the root assembles -- the stitched frame must be byte for byte the
    single-process frame of the whole input (lz4mtHipCompressFrame).  "ipc":
    packs pushed by device copies into the root's IPC-shared buffers (the
    multi-GPU default); "rccl": point-to-point over the group (gloo here)."""
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_streamed_rank, args=(r, 2, port, n, bid, cap, kind, q)) for r in range(2)]
    for p in procs:
        p.start()
    same, rounds, each = _qget(q, procs, 300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert same, (rounds, each)
    assert rounds >= 2


@pytest.mark.gpu
def test_bench_gpus3_strong_uneven_1mib_blocks():
    """Three ranks, ONE 0.25 GiB buffer of 1 MiB blocks (256 blocks: shards of
    86 / 85 / 85), streamed gather with the IPC push: the stitched frame is
    checked against every shard (dist.verify_stitched) and each rank decodes
    its scattered piece back to its source."""
    line = _bench("--gpus", "3", "--total-gib", "0.25", "--block-id", "6", "--steps", "1", "--warmup", "1",
                  "--no-cpu-baseline")
    assert line["n_gpus"] == 3 and line["scaling"] == "strong"
    assert line["config"]["bytes_total"] == 1 << 28 and line["config"]["block_bytes"] == 1 << 20
    assert line["gather"].startswith("streamed") and "ipc" in line["gather"]
    assert line["stitched_frame_ok"] is True and line["roundtrip_ok"] is True


def _nccl_world1(q, n, bid):
    """World size 1 over the nccl backend (RCCL allows one rank per device, so
    this is the most a one-GPU box can run): the whole N > 1 code path --
    control group, IPC transport setup, streamed gather, the device-walk
    scatter, the shard-by-shard stitched check -- on the device."""
    import torch.distributed as dist

    from lz4mt_amd import dist as D
    import lz4mt_amd as L
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
    try:
        sd = L.make_sd(bid, stream_checksum=False, block_checksum=True)
        src = L.gen_synthetic(n, seed=3)
        tr = D.IpcPushTransport(dev)
        st, sst = {}, {}
        full = D.compress_gather_streamed(src, sd, stats=st, transport=tr)
        tr.close()
        want = L.compress_frame(src, sd)
        same = full.numel() == want.numel() and bool(torch.equal(full, want))
        piece = D.scatter_frame(full, full.numel(), stats=sst)
        out, r = L.decompress_frame(piece)
        ok = D.verify_stitched(full, src, lambda f: L.decompress_frame(f)[0],
                               lambda t: L.xxh32_chunks(t, 1 << 20).to(torch.int64))
        q.put((dist.get_backend(), same, r == 0 and bool(torch.equal(out, src)), ok, sst.get("host_staged")))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_nccl_world1_streamed_gather_scatter_verify():
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_world1, args=(q, (40 << 20) + 4099, 7))
    p.start()
    backend, same, dec_ok, ok, staged = _qget(q, [p], 240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert backend == "nccl" and same and dec_ok and ok and staged is False


@pytest.mark.gpu
def test_bench_nccl_world1_distributed_path():
    """bench.py under torch.distributed.run with one rank, backend nccl set
    explicitly and the N > 1 path forced (LZ4MT_BENCH_DIST=1): the line
    reports the backend, the transport, the root's memory and the
    peer-access matrix, and every check passes."""
    env = dict(os.environ, LZ4MT_BENCH_BACKEND="nccl", LZ4MT_BENCH_DIST="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "1", "--gib", "0.25", "--steps", "1", "--warmup", "1", "--no-cpu-baseline"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    line = json.loads(lines[0])
    assert line["backend"] == "nccl" and line["transport"] == "ipc"
    assert line["stitched_frame_ok"] is True and line["roundtrip_ok"] is True
    assert line["gather"].startswith("streamed")
    assert line["root_memory"]["max_allocated_GiB"] > 0.25 and line["peer_access"][0][0] is True
    assert line["scatter_split_ms"]["host_staged"] is False


def _ipc_setup_rank(rank, world, port, corrupt, q):
    """One rank of an IpcPushTransport set-up on the shared test GPU (gloo):
    the root exports its receive buffers, the sender maps them (the root's GPU
    named by PCI bus id) and pushes the seeded pattern; the root checks it."""
    import torch.distributed as dist

    from lz4mt_amd import dist as D
    import lz4mt_amd as L
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if corrupt:
        os.environ["LZ4MT_AMD_IPC_CORRUPT"] = "1"
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=D.dist_timeout())
    try:
        sd = L.make_sd(7, stream_checksum=False, block_checksum=True)
        n = 96 << 20
        tr = D.IpcPushTransport(torch.device("cuda", 0))
        eng = D.HipShardEngine(torch.device("cuda", 0))
        try:
            D.prepare_transport(tr, eng, n, sd)
            res = ("ok", tr.kind)
            # the set-up is kept for the same layout: a streamed gather over it
            src = L.gen_synthetic(n, seed=77 + rank)
            full = D.compress_gather_streamed(src, sd, transport=tr, engine=eng)
            if rank == 0:   # whole 4 MiB blocks per shard: the frame of the concatenated shards
                want = L.compress_frame(torch.cat([L.gen_synthetic(n, seed=77), L.gen_synthetic(n, seed=78)]), sd)
                res = res + (full.numel() == want.numel() and bool(torch.equal(full, want)),)
            tr.close()
        except D.IpcSetupError as e:
            res = ("setup_error", str(e))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _run_two(target, *args, timeout=240):
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, 2, port, *args, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(_qget(q, procs, timeout) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


@pytest.mark.gpu
def test_ipc_setup_pattern_check_passes():
    """the IPC set-up proves the push end to end (seeded
    pattern, XXH32 per 1 MiB compared on the root) and reports the receive
    buffers' memory kind; a streamed gather then runs over it."""
    got = _run_two(_ipc_setup_rank, False)
    assert got[0][0] == "ok" and got[1][0] == "ok", got
    assert got[0][1] == "uncached"   # the push takes uncached receive buffers or none
    assert got[0][2] is True


@pytest.mark.gpu
def test_ipc_setup_corrupt_pattern_fails_on_every_rank():
    """A pattern that does not arrive intact (LZ4MT_AMD_IPC_CORRUPT=1 flips a
    byte after the sender's digests) raises IpcSetupError on BOTH ranks."""
    got = _run_two(_ipc_setup_rank, True)
    assert got[0][0] == "setup_error" and got[1][0] == "setup_error", got
    assert "pattern check failed" in got[0][1]


@pytest.mark.gpu
def test_bench_corrupt_ipc_falls_back_to_rccl():
    """bench.py at N = 2 with a forced-corrupt pattern: every rank takes the
    RCCL (here: gloo point-to-point) transport together, the line says so,
    and the stitched frame is still right."""
    env_extra = {"LZ4MT_AMD_IPC_CORRUPT": "1"}
    old = {k: os.environ.get(k) for k in env_extra}
    os.environ.update(env_extra)
    try:
        line = _bench("--gpus", "2", "--gib", "0.25", "--steps", "1", "--warmup", "0", "--no-cpu-baseline")
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert line["transport"].startswith("rccl (IPC setup failed") and "pattern check failed" in line["transport"]
    assert line["stitched_frame_ok"] is True and line["roundtrip_ok"] is True


def _bench_fail(fault, deadline=300, timeout=300):
    """bench.py --gpus 2 (gloo, both ranks on the test GPU) with a fault
    injected by LZ4MT_BENCH_FAULT: returns (exit code, the one JSON line,
    wall seconds)."""
    import time
    env = dict(os.environ, LZ4MT_BENCH_BACKEND="gloo", LZ4MT_BENCH_FAULT=fault,
               LZ4MT_BENCH_DEADLINE_S=str(deadline))
    env.pop("WORLD_SIZE", None)
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--gib", "0.25", "--steps", "1",
                        "--warmup", "0", "--no-cpu-baseline"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    return r.returncode, json.loads(lines[0]), time.monotonic() - t0


@pytest.mark.gpu
@pytest.mark.parametrize("fault,stage", [("setup:1", "setup"), ("gather:1", "step"), ("step:0", "step")])
def test_bench_n2_failure_is_one_json_line(fault, stage):
    """an exception on any rank at N > 1 -- at set-up,
    or mid-step between the gather and the scatter while the root waits in a
    collective -- ends the run non-zero with ONE JSON line on rank 0 naming
    the stage, the transport and the error, well within the deadline."""
    rc, line, dt = _bench_fail(fault)
    assert rc != 0
    assert line["status"] == "failed" and line["value"] is None and line["n_gpus"] == 2
    assert line["stage"] == stage and line["failed_rank"] == int(fault.split(":")[1])
    assert line["transport"] == "ipc" and "injected fault" in line["error"]
    assert line["elapsed_s"] < 120 and dt < 240


@pytest.mark.gpu
def test_bench_n2_hang_ends_at_the_deadline():
    """A rank that hangs mid-step (no exception, no collective error) is
    ended by the deadline: the same one line, 'deadline exceeded'."""
    rc, line, dt = _bench_fail("gather:1:hang", deadline=45)
    assert rc != 0
    assert line["status"] == "failed" and line["stage"] == "step" and "deadline exceeded" in line["error"]
    assert line["elapsed_s"] < 90 and dt < 240


@pytest.mark.gpu
def test_shard_call_order_is_enforced():
    """an encode into a workspace not reset since its last encode,
    or a pack from a workspace never encoded since its reset, is BAD_ARG."""
    import ctypes

    import lz4mt_amd as L
    n = 8 << 20
    sd = L.make_sd(7, stream_checksum=False, block_checksum=True)
    src = L.gen_synthetic(n, seed=5)
    ws = torch.zeros(L.lib.lz4mtHipShardWorkspaceSize(n, ctypes.byref(sd)), dtype=torch.uint8, device="cuda")
    pk = torch.empty(L.shard_pack_bound(n, sd, 64 << 10), dtype=torch.uint8, device="cuda")

    def enc():
        return L.lib.lz4mtHipShardEncode(ctypes.c_void_p(src.data_ptr()), n, ctypes.byref(sd),
                                         ctypes.c_void_p(ws.data_ptr()), ws.numel(), None)

    def pack():
        return L.lib.lz4mtHipShardPack(ctypes.c_void_p(src.data_ptr()), n, ctypes.byref(sd),
                                       ctypes.c_void_p(ws.data_ptr()), ws.numel(), ctypes.c_void_p(pk.data_ptr()),
                                       pk.numel(), 64 << 10, 0, None)
    BAD = int(L.Result.BAD_ARG)
    assert enc() == BAD                      # fresh workspace, never reset
    assert pack() == BAD
    assert L.lib.lz4mtHipShardReset(n, ctypes.byref(sd), ctypes.c_void_p(ws.data_ptr()), ws.numel(), None) == 0
    assert pack() == BAD                     # reset but not encoded
    assert enc() == 0
    assert pack() == 0
    assert enc() == BAD                      # a second encode without a reset
    torch.cuda.synchronize()
