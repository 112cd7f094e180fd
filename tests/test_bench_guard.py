"""bench.py's N > 1 runs end bounded and say why, on CPU.

tests/guard_worker.py runs bench.RunGuard over a gloo group of 2 or 3 ranks
launched by torch.distributed.run, exactly as bench.py's ranks do.  A fault
injected on one rank in one stage (LZ4MT_BENCH_FAULT) must end the whole run
non-zero with ONE JSON line on stdout naming that stage, the transport and
the error -- also when the failing rank is not rank 0 and rank 0 sits in a
collective waiting for it, and when a rank hangs instead of failing (the
deadline).  The GPU versions (bench.py itself on the device) are in
tests/test_gpu_dist.py."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, fault=None, deadline=60, timeout=150):
    env = dict(os.environ, LZ4MT_BENCH_DEADLINE_S=str(deadline))
    env.pop("LZ4MT_BENCH_FAULT", None)
    if fault:
        env["LZ4MT_BENCH_FAULT"] = fault
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()),
                        os.path.join(ROOT, "tests", "guard_worker.py")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, lines, time.monotonic() - t0


def test_guard_success_prints_one_line():
    r, lines, _ = _run(2)
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1 and json.loads(lines[0])["value"] == 1.0


@pytest.mark.parametrize("fault,stage", [("setup:1", "setup"), ("gather:1", "step"), ("setup:0", "setup"),
                                         ("check:2", "check")])
def test_guard_failure_is_one_line_naming_the_stage(fault, stage):
    world = 3 if fault.endswith(":2") else 2
    r, lines, dt = _run(world, fault)
    assert r.returncode != 0
    assert len(lines) == 1, (r.stdout[-2000:], r.stderr[-3000:])
    line = json.loads(lines[0])
    assert line["status"] == "failed" and line["value"] is None and line["n_gpus"] == world
    assert line["stage"] == stage and line["transport"] == "ipc"
    assert line["failed_rank"] == int(fault.split(":")[1])
    assert "injected fault" in line["error"]
    assert dt < 60, dt   # bounded well below the deadline: a failure is reported at once


def test_guard_hang_ends_at_the_deadline():
    r, lines, dt = _run(2, "gather:1:hang", deadline=12)
    assert r.returncode != 0
    assert len(lines) == 1, (r.stdout[-2000:], r.stderr[-3000:])
    line = json.loads(lines[0])
    assert line["status"] == "failed" and line["stage"] == "step"
    assert "deadline exceeded" in line["error"]
    assert 12 <= line["elapsed_s"] < 40 and dt < 90
