# A/B: speculative round trip (issued from the table read, before the readback / predecessor resolution)
set -euo pipefail
out=gpurun_out/r02at
mkdir -p $out
export TMPDIR=/tmp
bash tools/ab.sh > $out/ab.txt 2>&1
bash tools/ab.sh >> $out/ab.txt 2>&1
LZ4MT_AMD_LIB=exp_libs/specB1.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py tests/test_gpu_bd.py -m gpu > $out/tests_spec1.log 2>&1
