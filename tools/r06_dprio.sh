#!/bin/bash
# round 6: the SIMD-mate priority in the decoder (decode_block, blocks >= 1 MiB)
# vs the same build without it (LZ4MT_NO_DEC_PRIO): parity screen, kernel
# times B7 / B6 / B5, per-block end times of k_decode at B7
set -uo pipefail
out=gpurun_out/r06x
mkdir -p "$out"
export TMPDIR=/tmp BT_OUT=$out
LZ4MT_AMD_LIB=exp_libs/dprio.so timeout -k 10 300 python3 -u tools/abparity.py 2>&1 | grep -v amdgpu | tee "$out/parity.txt" || exit 1
LZ4MT_AMD_LIB=exp_bt/blktime_prio.so timeout -k 10 200 python3 -u tools/blocktimes.py 7 --decode 2>&1 | grep -v amdgpu > "$out/bt_dec_b7.txt" || exit 1
for pass in 1 2 3; do
  for b in 7 6 5; do
    BID=$b bash tools/ab.sh 2>&1 | tee -a "$out/ab_b$b.txt"
  done
done
