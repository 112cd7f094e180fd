#!/bin/bash
# round 6: the sequence layout's remainders mod 256 without a multiply
# (SeqLayout<R8>) on the small-block encoders only (r8small, the default:
# k_encode16 / k_encode_p17), on every encoder (r8all), on none (base);
# B4 / B5 / B7, parity screen
set -uo pipefail
out=gpurun_out/r06q
mkdir -p "$out"
export TMPDIR=/tmp
for v in r8small r8all; do
  LZ4MT_AMD_LIB=exp_libs/$v.so timeout -k 10 300 python3 -u tools/abparity.py 2>&1 | grep -v amdgpu | tee -a "$out/parity.txt" || exit 1
done
for pass in 1 2; do
  BID=4 bash tools/ab.sh 2>&1 | tee -a "$out/ab_b4.txt"
  BID=5 bash tools/ab.sh 2>&1 | tee -a "$out/ab_b5.txt"
  bash tools/ab.sh 2>&1 | tee -a "$out/ab_b7.txt"
done
