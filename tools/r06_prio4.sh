#!/bin/bash
# round 6: SIMD-mate priority variants (cuprio: rank among the CU's 8 waves;
# s6 / s8: checks every 1/64 / 1/256 of the block) vs the product, B7 / B6;
# the decoder's per-block end times (is there the same younger-wave tail?)
set -uo pipefail
out=gpurun_out/r06w
mkdir -p "$out"
export TMPDIR=/tmp BT_OUT=$out
LZ4MT_AMD_LIB=exp_bt/blktime_prio.so timeout -k 10 200 python3 -u tools/blocktimes.py 7 --decode 2>&1 | grep -v amdgpu > "$out/bt_dec_b7.txt" || exit 1
LZ4MT_AMD_LIB=exp_libs/cuprio.so timeout -k 10 300 python3 -u tools/abparity.py 2>&1 | grep -v amdgpu | tee "$out/parity.txt" || exit 1
for pass in 1 2; do
  for b in 7 6; do
    BID=$b bash tools/ab.sh 2>&1 | tee -a "$out/ab_b$b.txt"
  done
done
