#!/bin/bash
# GPU side of an HC A/B: tools/hctime.py for every exp_libs/*.so twice, then the HC parity tests against exp_libs/$1.so
# usage (on the box): bash tools/abhc.sh <name> <tag>
set -euo pipefail
name=$1; tag=$2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
  for f in exp_libs/*.so; do
    LZ4MT_AMD_LIB=$f timeout -k 10 200 python3 -u tools/hctime.py 2>&1 | grep -v amdgpu >> $out/ab.txt
  done
done
LZ4MT_AMD_LIB=exp_libs/$name.so timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_hc.py tests/test_gpu_bd_hc.py -m gpu > $out/tests.log 2>&1
