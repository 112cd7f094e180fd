#!/bin/bash
# round 6: encoder quarter-rate ops (LZ4MT_EXP_REM8: the sequence layout's
# remainders mod 256 without a multiply; LZ4MT_EXP_HASH24: the hash5 product
# as one 32x32 mad + two 24-bit multiplies) vs base, B7 / B6 / B5, parity
# screen of every variant
set -uo pipefail
out=gpurun_out/r06p
mkdir -p "$out"
export TMPDIR=/tmp
for v in rem8 hash24 rh; do
  LZ4MT_AMD_LIB=exp_libs/$v.so timeout -k 10 300 python3 -u tools/abparity.py 2>&1 | grep -v amdgpu | tee -a "$out/parity.txt" || exit 1
done
for pass in 1 2; do
  bash tools/ab.sh 2>&1 | tee -a "$out/ab_b7.txt"
  BID=6 bash tools/ab.sh 2>&1 | tee -a "$out/ab_b6.txt"
done
BID=5 bash tools/ab.sh 2>&1 | tee -a "$out/ab_b5.txt"
