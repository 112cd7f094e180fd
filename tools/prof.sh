#!/bin/bash
# Profiles for one round: kernel-trace stats of the bench command, then HBM
# counters (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md
# "rocprofv3 PMC slots") on one 8 GiB compress+decompress (tools/kprof.py).
# usage: tools/prof.sh <tag>      (run from the repo root on the GPU box)
set -euo pipefail
tag=${1:-r01}
out=gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$out/trace" -o trace -- \
    python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > "$out/bench.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -T -f csv -d "$out/fetch" -o fetch -- \
    python3 tools/kprof.py 8 > "$out/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -T -f csv -d "$out/write" -o write -- \
    python3 tools/kprof.py 8 > "$out/write.log" 2>&1
echo done
