#!/bin/bash
# round 6: the encoder object's compiler schedule re-swept on the trimmed
# window (mmc = the product's max-memory-clause without memory-op clustering)
set -uo pipefail
out=gpurun_out/r06r
mkdir -p "$out"
export TMPDIR=/tmp
for pass in 1 2; do
  bash tools/ab.sh 2>&1 | tee -a "$out/ab_b7.txt"
  BID=6 bash tools/ab.sh 2>&1 | tee -a "$out/ab_b6.txt"
done
