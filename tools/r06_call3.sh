#!/bin/bash
# round 6: IPC memory kinds by size (the B5 gather test got no uncached
# buffer), then the streamed e2e rate at 8 / 4 / 2 waves per CU (B7) and at
# every block size with the default
set -uo pipefail
out=gpurun_out/r06c
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 120 python3 -u tools/probe/ipc_kinds.py 2>&1 | tee "$out/ipc_kinds.txt" || exit 1
for w in 8 4 2; do
  LZ4MT_AMD_STREAM_WAVES_PER_CU=$w timeout -k 10 300 python3 -u tools/e2e.py 8 7 > "$out/e2e_b7_w$w.txt" 2>&1 \
      || { tail -20 "$out/e2e_b7_w$w.txt"; exit 1; }
  grep e2e "$out/e2e_b7_w$w.txt" | sed "s/^/B7 waves_per_cu=$w: /"
done
for b in 4 5 6; do
  timeout -k 10 300 python3 -u tools/e2e.py 8 $b > "$out/e2e_b${b}.txt" 2>&1 || { tail -20 "$out/e2e_b$b.txt"; exit 1; }
  grep e2e "$out/e2e_b$b.txt" | sed "s/^/B$b: /"
  LZ4MT_AMD_STREAM=0 timeout -k 10 300 python3 -u tools/e2e.py 8 $b > "$out/e2e_b${b}_batch.txt" 2>&1 \
      || { tail -20 "$out/e2e_b${b}_batch.txt"; exit 1; }
  grep e2e "$out/e2e_b${b}_batch.txt" | sed "s/^/B$b batch: /"
done
