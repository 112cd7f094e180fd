#!/bin/bash
# round 6: the streamed-engine tests on the monitor-relaunch build, the
# streamed e2e at B4 / B6 / B7 on it, then the encoder interference and
# block-XXH32-beside-the-encode A/Bs
set -uo pipefail
out=gpurun_out/r06h
mkdir -p "$out"
export TMPDIR=/tmp
bash tools/gpu_round.sh r06h tstream || exit 1
for b in 4 6 7; do
  timeout -k 10 300 python3 -u tools/e2e.py 8 $b > "$out/e2e_b${b}.txt" 2>&1 || { tail -20 "$out/e2e_b$b.txt"; exit 1; }
  grep e2e "$out/e2e_b$b.txt" | sed "s/^/B$b: /"
done
bash tools/gpu_round.sh r06h interf follow
