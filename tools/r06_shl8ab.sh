#!/bin/bash
# round 6: encoder trim (LZ4MT_EXP_SHL8: 255*ext in the sequence layout as
# (ext<<8)-ext, full-rate shifts instead of a quarter-rate multiply) vs base,
# B7 and B6, parity screen of the variant
set -uo pipefail
out=gpurun_out/r06l
mkdir -p "$out"
export TMPDIR=/tmp
LZ4MT_AMD_LIB=exp_libs/shl8.so timeout -k 10 300 python3 -u tools/abparity.py 2>&1 | grep -v amdgpu | tee "$out/parity.txt"
for pass in 1 2; do
  bash tools/ab.sh 2>&1 | tee -a "$out/ab_b7.txt"
  BID=6 bash tools/ab.sh 2>&1 | tee -a "$out/ab_b6.txt"
done
