# LZ4-HC levels 10..12 on the GPU: HC parity tests (golden blocks at 3..12, fuzz, frames, callback API)
set -euo pipefail
out=gpurun_out/r02ba
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_hc.py -m gpu > $out/tests.log 2>&1
