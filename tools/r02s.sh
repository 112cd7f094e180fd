set -euo pipefail
out=gpurun_out/r02s
mkdir -p $out
export TMPDIR=/tmp LZ4MT_AMD_HASH_STATS=1
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --stream-checksum --no-cpu-baseline > $out/bench_sck.json 2>$out/sck.err
grep "host hash" $out/sck.err | tail -4
