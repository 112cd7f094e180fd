#!/bin/bash
# round 6: encoder instruction trims (LZ4MT_EXP_TRIM: the sequence layout
# reuses the window's extension lengths, do-while byte rounds, the hash-input
# read without an else branch) vs base, B7 and B6, parity screen of the variant
set -uo pipefail
out=gpurun_out/r06k
mkdir -p "$out"
export TMPDIR=/tmp
LZ4MT_AMD_LIB=exp_libs/trim.so timeout -k 10 300 python3 -u tools/abparity.py 2>&1 | grep -v amdgpu | tee "$out/parity.txt"
for pass in 1 2; do
  bash tools/ab.sh 2>&1 | tee -a "$out/ab_b7.txt"
  BID=6 bash tools/ab.sh 2>&1 | tee -a "$out/ab_b6.txt"
done
