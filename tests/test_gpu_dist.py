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
        data = bytearray(oracle.gen_synthetic(n, 42))
        rnd = oracle.gen_random(n, 5)
        for s in range(0, n, 5 << 20):
            data[s:s + 1_200_000] = rnd[s:s + 1_200_000]
        bm = 1 << (8 + 2 * bid)
        off, ln, _, _ = D.shard_blocks(n, bm, world, rank)
        src = torch.frombuffer(bytearray(data[off:off + ln]), dtype=torch.uint8).cuda()
        sd = L.make_sd(bid, stream_checksum=False, block_checksum=True)
        st = {}
        tr = D.IpcPushTransport(torch.device("cuda", 0)) if kind == "ipc" else D.RcclTransport()
        full = None
        for _ in range(2):   # twice: the IPC buffers are set up once and reused
            full = D.compress_gather_streamed(src, sd, per_block_cap=cap, stats=st, min_round_s=0.0005,
                                              transport=tr)
        tr.close()
        if rank == 0:
            want = L.compress_frame(torch.frombuffer(data, dtype=torch.uint8).cuda(), sd)
            q.put((full.numel() == want.numel() and bool(torch.equal(full, want)), st["rounds"], full.numel()))
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
    same, rounds, size = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert same, (rounds, size)
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
