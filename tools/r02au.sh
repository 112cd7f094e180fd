# results refresh with the current build: block-size sweep (configs[4]), 32 GiB decompress-only
# (configs[2]), -BD B7/B4, HC9, default flags
set -euo pipefail
out=gpurun_out/r02au
mkdir -p $out
export TMPDIR=/tmp
for b in 4 5 6; do
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --block-id $b --no-cpu-baseline > $out/sweep_b$b.json 2>$out/sweep_b$b.err
done
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --gib 32 --decompress-only --no-cpu-baseline > $out/dec32.json 2>$out/dec32.err
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --block-dependent --no-cpu-baseline > $out/bd7.json 2>$out/bd7.err
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --block-id 4 --block-dependent --no-cpu-baseline > $out/bd4.json 2>$out/bd4.err
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --level 9 --no-cpu-baseline > $out/hc9.json 2>$out/hc9.err
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --stream-checksum --no-cpu-baseline > $out/sck.json 2>$out/sck.err
