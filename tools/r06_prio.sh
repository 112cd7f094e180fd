#!/bin/bash
# round 6: the encoder's tail -- per-block end times (LZ4MT_EXP_BLKTIME) with
# and without the SIMD-pair priority (LZ4MT_EXP_PRIO), kernel A/B at B7 / B6
set -uo pipefail
out=gpurun_out/r06t
mkdir -p "$out"
export TMPDIR=/tmp BT_OUT=$out
for v in blktime blkprio; do
  LZ4MT_AMD_LIB=exp_libs/$v.so timeout -k 10 200 python3 -u tools/blocktimes.py 7 2>&1 | grep -v amdgpu > "$out/bt_${v}_b7.txt" || exit 1
  LZ4MT_AMD_LIB=exp_libs/$v.so timeout -k 10 200 python3 -u tools/blocktimes.py 6 2>&1 | grep -v amdgpu > "$out/bt_${v}_b6.txt" || exit 1
done
LZ4MT_AMD_LIB=exp_libs/prio.so timeout -k 10 300 python3 -u tools/abparity.py 2>&1 | grep -v amdgpu | tee "$out/parity.txt" || exit 1
for pass in 1 2; do
  bash tools/ab.sh 2>&1 | tee -a "$out/ab_b7.txt"
  BID=6 bash tools/ab.sh 2>&1 | tee -a "$out/ab_b6.txt"
done
