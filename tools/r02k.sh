set -euo pipefail
out=gpurun_out/r02k
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$out/bd4" -o trace -- \
    python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --gib 1 --block-dependent --block-id 4 > "$out/bd4.log" 2>&1
find $out -name "*kernel_stats.csv" | head
