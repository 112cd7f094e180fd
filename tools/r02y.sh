set -euo pipefail
out=gpurun_out/r02y
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py -k "known_answers_large" > $out/pytest.log 2>&1
tail -3 $out/pytest.log
