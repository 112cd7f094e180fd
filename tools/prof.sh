#!/bin/bash
# Profiles for one round: kernel-trace stats of the bench command, then HBM
# counters (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md
# "rocprofv3 PMC slots") on one 8 GiB compress+decompress of App. F input
# (tools/kprof.py 8) and of random bytes (the FETCH_SIZE calibration).
# usage: tools/prof.sh <tag>      (run from the repo root on the GPU box)
set -euo pipefail
tag=${1:-r02}
out=gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$out/trace" -o trace -- \
    python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > "$out/bench.log" 2>&1
for input in appf random; do
    flag=""; [ "$input" = random ] && flag="--random"
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -T -f csv -d "$out/fetch_$input" -o fetch -- \
        python3 tools/kprof.py 8 $flag > "$out/fetch_$input.log" 2>&1
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -T -f csv -d "$out/write_$input" -o write -- \
        python3 tools/kprof.py 8 $flag > "$out/write_$input.log" 2>&1
done
echo done
