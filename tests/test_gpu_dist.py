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
    # the stitched frame is ONE frame of the whole 2 x 0.25 GiB stream: header + records + EOS
    assert line["stitched_frame_bytes"] > line["frame_bytes"]


@pytest.mark.gpu
def test_bench_gpus2_strong_scaling_one_buffer():
    # 0.5 GiB of 4 MiB blocks = 128 blocks, 64 per rank: the two shards are
    # consecutive pieces of ONE App. F buffer, stitched into one frame
    line = _bench("--gpus", "2", "--total-gib", "0.5", "--steps", "1", "--warmup", "0", "--no-cpu-baseline")
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["bytes_total"] == 1 << 29
    assert line["stitched_frame_ok"] is True and line["roundtrip_ok"] is True
