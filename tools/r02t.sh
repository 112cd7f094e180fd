set -euo pipefail
out=gpurun_out/r02t
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu.py -k "compress or frames_golden or known_answers" > $out/pytest.log 2>&1
tail -1 $out/pytest.log
for i in 1 2; do timeout -k 10 300 bash tools/ab.sh; done > $out/ab.txt 2>&1
grep -v amdgpu $out/ab.txt
