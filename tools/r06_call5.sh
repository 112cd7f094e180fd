#!/bin/bash
# round 6: B4 4-bit-tag table A/B, then k_encode_p17
# traffic at 11 vs 8 waves per CU (item 7)
set -uo pipefail
out=gpurun_out/r06f
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/t4_ab.py 2>&1 | tee "$out/t4_ab.txt"
[ "${PIPESTATUS[0]}" = 0 ] || echo "t4_ab: nonzero exit"
bash tools/r06_b5occ.sh
