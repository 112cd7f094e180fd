# final-build sweep: configs[4] block sizes, configs[2] decompress-only, default flags, HC level 9, -BD B7
set -euo pipefail
out=gpurun_out/r03x; mkdir -p $out
run() { name=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > $out/$name.json 2> $out/$name.err; echo "$name $(cut -c1-400 $out/$name.json)"; }
run b4 --block-id 4 --steps 5 --warmup 2
run b5 --block-id 5 --steps 5 --warmup 2
run b6 --block-id 6 --steps 5 --warmup 2
run dec32 --gib 32 --decompress-only --steps 3 --warmup 1
run sck --stream-checksum --steps 3 --warmup 1
run hc9 --level 9 --steps 2 --warmup 1
run bd7 --block-dependent --steps 2 --warmup 1
