#!/bin/bash
# round 6: k_encode_p17's counter traffic at 256 KiB
# blocks against its occupancy: 11 waves per CU (no pad) vs 8 (LDS padded to
# 20 KiB per wave, LZ4MT_AMD_ENC_LDS_PAD=5888) -- FETCH_SIZE and WRITE_SIZE in
# separate passes, kernel time from the same traces
set -uo pipefail
out=gpurun_out/r06d
mkdir -p "$out"
export TMPDIR=/tmp
for pad in 0 5888; do
  for c in FETCH_SIZE WRITE_SIZE; do
    n=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
    LZ4MT_AMD_ENC_LDS_PAD=$pad timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c -T -f csv \
        -d "$out/pad$pad/${n}_appf" -o $n -- python3 tools/kprof.py 8 --bid=5 > "$out/pad${pad}_$n.log" 2>&1 \
        || { echo "pad $pad $c failed"; tail -5 "$out/pad${pad}_$n.log"; exit 1; }
    echo "pad $pad $c ok"
  done
done
