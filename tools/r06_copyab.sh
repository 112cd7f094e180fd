#!/bin/bash
# round 6: the memory binding's copy split (lz4mtMemBind read/write through
# par_copy) A/B at 256 KiB .. 4 MiB blocks: default (split >= 2 MiB into
# 1 MiB pieces) vs split >= 512 KiB into 256 KiB pieces vs >= 256 KiB into 128 KiB
set -uo pipefail
out=${OUT:-gpurun_out/r06j}
mkdir -p "$out"
export TMPDIR=/tmp
cfgs=("2048 1024" "512 256" "256 128")
[ -n "${CFGS:-}" ] && IFS=, read -ra cfgs <<< "$CFGS"   # e.g. CFGS="2048 1024,512 256"
for cfg in "${cfgs[@]}"; do
  set -- $cfg
  for b in 5 6 7; do
    LZ4MT_AMD_COPY_MIN_KIB=$1 LZ4MT_AMD_COPY_PIECE_KIB=$2 timeout -k 10 300 python3 -u tools/e2e.py 8 $b \
        > "$out/e2e_b${b}_min$1_piece$2.txt" 2>&1 || { tail -20 "$out/e2e_b${b}_min$1_piece$2.txt"; exit 1; }
    grep "Sx -BX" "$out/e2e_b${b}_min$1_piece$2.txt" | sed "s/^/min $1 KiB piece $2 KiB: /"
  done
done
