# LZ4-HC optimal parser benches (1 GiB App. F, 4 MiB and 256 KiB blocks) with the HC CPU baseline
set -euo pipefail
out=gpurun_out/r02bb
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --gib 1 --steps 1 --warmup 1 --level 10 > $out/hc10.json 2>$out/hc10.err
timeout -k 10 400 python3 bench.py --gib 1 --steps 1 --warmup 1 --level 12 > $out/hc12.json 2>$out/hc12.err
timeout -k 10 400 python3 bench.py --gib 1 --steps 1 --warmup 1 --level 12 --block-id 5 --no-cpu-baseline > $out/hc12_b5.json 2>$out/hc12_b5.err
