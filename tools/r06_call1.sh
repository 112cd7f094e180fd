#!/bin/bash
# round 6, first box: the changed GPU tests (streamed engines with write-side
# parking, N > 1 failure lines) and the streamed e2e rate at 8 / 4 / 2 waves per CU
set -euo pipefail
out=gpurun_out/r06a
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_stream.py tests/test_gpu_dist.py > "$out/pytest.log" 2>&1 || { tail -40 "$out/pytest.log"; exit 1; }
tail -3 "$out/pytest.log"
for w in 8 4 2; do
  LZ4MT_AMD_STREAM_WAVES_PER_CU=$w timeout -k 10 300 python3 tools/e2e.py 8 7 > "$out/e2e_w$w.txt" 2>&1 \
      || { tail -20 "$out/e2e_w$w.txt"; exit 1; }
  grep e2e "$out/e2e_w$w.txt" | sed "s/^/waves_per_cu=$w: /"
done
