set -euo pipefail
mkdir -p gpurun_out/r02j
export TMPDIR=/tmp
export LZ4MT_AMD_BD_STATS=1
timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --gib 1 --block-dependent --no-cpu-baseline > gpurun_out/r02j/bench_bd.json 2>&1
timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --gib 1 --block-dependent --block-id 4 --no-cpu-baseline > gpurun_out/r02j/bench_bd4.json 2>&1
timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --gib 1 --block-dependent --block-id 5 --no-cpu-baseline > gpurun_out/r02j/bench_bd5.json 2>&1
grep -h "lz4mt -BD" gpurun_out/r02j/*.json
