set -euo pipefail
out=gpurun_out/r02u
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/ > $out/pytest.log 2>&1
tail -2 $out/pytest.log
timeout -k 10 600 python3 -u tools/e2e.py 8 7 --file /dev/shm > $out/e2e_file.txt 2>&1
grep -v amdgpu $out/e2e_file.txt
