# -BD fast path at 8 GiB for 64 KiB .. 1 MiB blocks, with the rounds' stats
set -euo pipefail
out=gpurun_out/r02al
mkdir -p $out
export TMPDIR=/tmp LZ4MT_AMD_BD_STATS=1
for b in 4 5 6; do
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --block-id $b --block-dependent --no-cpu-baseline > $out/bd$b.json 2>$out/bd$b.err
done
