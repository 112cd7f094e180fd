"""A rank of bench.py's N > 1 failure path without a GPU (tests/test_bench_guard.py).

Launched by torch.distributed.run on CPU: every rank makes bench.RunGuard
exactly as bench.py does, joins a gloo group, then walks bench.py's stages
with a collective in each -- so a fault injected on one rank
(LZ4MT_BENCH_FAULT) leaves the others blocked in a collective, as a failed
GPU rank would.  Rank 0 prints bench.py's result line when nothing fails."""
import datetime
import json
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    guard = bench.RunGuard(rank, world, world, enabled=True)
    try:
        guard.enter("init")
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=guard.deadline_s + 60))
        guard.transport = "ipc"
        for stage in ("input", "setup", "step"):
            guard.enter(stage)
            # bench.py connects its control group with fd 1 redirected to
            # stderr: a failure line printed meanwhile must still reach stdout
            with bench.stdout_to_stderr():
                dist.barrier()
        guard.enter("step", point="gather")
        t = torch.ones(4)
        dist.all_reduce(t)
        for stage in ("check", "report"):
            guard.enter(stage)
            dist.barrier()
        if rank == 0 and guard.succeeded(True):
            print(json.dumps({"metric": bench.METRIC, "value": 1.0, "n_gpus": world}), flush=True)
        elif rank != 0:
            guard.succeeded(True)
        dist.destroy_process_group()
        guard.cleanup()
    except BaseException as e:   # noqa: B902 -- as bench.main
        traceback.print_exc(file=sys.stderr)
        guard.failed(f"{type(e).__name__}: {e}")


if __name__ == "__main__":
    main()
