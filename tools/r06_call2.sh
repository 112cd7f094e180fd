#!/bin/bash
# round 6: the B5 streamed-gather test alone (it stalled in r06a), output unbuffered
set -uo pipefail
out=gpurun_out/r06b
mkdir -p "$out"
export TMPDIR=/tmp
export PYTHONFAULTHANDLER=1
timeout -k 10 200 python3 -u -m pytest -m gpu -x -v -s --timeout 100 --timeout-method thread \
    "tests/test_gpu_dist.py::test_streamed_gather_on_device[12583011-5-65536-ipc]" \
    "tests/test_gpu_dist.py::test_streamed_gather_on_device[12583011-5-65536-rccl]" 2>&1 | tee "$out/pytest.log"
echo "rc=$?"
