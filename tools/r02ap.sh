# A/B: forward-count words per round trip (63 = current, 32, 16); parity of the 16-lane build
set -euo pipefail
out=gpurun_out/r02ap
mkdir -p $out
export TMPDIR=/tmp
bash tools/ab.sh > $out/ab.txt 2>&1
bash tools/ab.sh >> $out/ab.txt 2>&1
LZ4MT_AMD_LIB=exp_libs/k16.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py -m gpu > $out/tests_k16.log 2>&1
