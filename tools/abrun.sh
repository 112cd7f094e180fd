#!/bin/bash
# GPU side of an A/B: timings of every exp_libs/*.so twice, then the parity tests against exp_libs/$1.so
# usage (on the box): bash tools/abrun.sh <name> <tag> [test files...]
set -euo pipefail
name=$1; tag=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
bash tools/ab.sh > $out/ab.txt 2>&1
bash tools/ab.sh >> $out/ab.txt 2>&1
tests="${*:-tests/test_gpu.py}"
LZ4MT_AMD_LIB=exp_libs/$name.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread $tests -m gpu > $out/tests.log 2>&1
