#!/bin/bash
# round 6: the product's SIMD-mate priority (encode_block_v5, byU32 blocks
# >= 1 MiB) vs the same build without it (LZ4MT_NO_SIMD_PRIO): parity screen,
# kernel times B7 / B6 / B5 / B4, per-block end times at B7 (LZ4MT_EXP_BLKTIME)
set -uo pipefail
out=gpurun_out/r06v
mkdir -p "$out"
export TMPDIR=/tmp BT_OUT=$out
LZ4MT_AMD_LIB=exp_libs/prio.so timeout -k 10 300 python3 -u tools/abparity.py 2>&1 | grep -v amdgpu | tee "$out/parity.txt" || exit 1
for v in base prio; do
  LZ4MT_AMD_LIB=exp_bt/blktime_$v.so timeout -k 10 200 python3 -u tools/blocktimes.py 7 2>&1 | grep -v amdgpu > "$out/bt_${v}_b7.txt" || exit 1
done
for pass in 1 2; do
  for b in 7 6 5 4; do
    BID=$b bash tools/ab.sh 2>&1 | tee -a "$out/ab_b$b.txt"
  done
done
