set -euo pipefail
out=gpurun_out/r02q
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_bd.py > $out/pytest.log 2>&1
tail -2 $out/pytest.log
