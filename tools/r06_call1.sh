#!/bin/bash
# round 6: the changed GPU tests (N > 1 failure lines, IPC set-up, streamed
# engines with write-side parking and every block size)
set -euo pipefail
out=gpurun_out/r06e
mkdir -p "$out"
export TMPDIR=/tmp
export LZ4MT_AMD_IPC_TRACE=1
timeout -k 10 1000 python3 -u -m pytest -m gpu -x -v --timeout 280 --timeout-method thread \
    tests/test_gpu_dist.py tests/test_gpu_stream.py tests/test_gpu_configs.py 2>&1 | tee "$out/pytest.log" | grep -E "PASSED|FAILED|ERROR|passed|failed" || true
tail -3 "$out/pytest.log"
