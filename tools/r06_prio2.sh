#!/bin/bash
# round 6: SIMD-mate issue priority for the encoder's tail -- pair (p1) vs
# rank among the SIMD's waves (p2; check every blen >> 7, s6 / s8: >> 6 / >> 8)
# vs base, B7 / B6 / B5 / B4, parity screen of p2
set -uo pipefail
out=gpurun_out/r06u
mkdir -p "$out"
export TMPDIR=/tmp
LZ4MT_AMD_LIB=exp_libs/p2.so timeout -k 10 300 python3 -u tools/abparity.py 2>&1 | grep -v amdgpu | tee "$out/parity.txt" || exit 1
for pass in 1 2; do
  for b in 7 6 5 4; do
    BID=$b bash tools/ab.sh 2>&1 | tee -a "$out/ab_b$b.txt"
  done
done
