set -euo pipefail
out=gpurun_out/r02ab
mkdir -p $out
export TMPDIR=/tmp LZ4MT_AMD_BD_STATS=1
run() { timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --gib 1 --block-dependent --block-id $1 --no-cpu-baseline > $out/$2.json 2>$out/$2.err; }
LZ4MT_AMD_BD_WARM_KIB=0 run 7 b7_w0
LZ4MT_AMD_BD_WARM_KIB=256 run 7 b7_w256
LZ4MT_AMD_BD_WARM_KIB=512 run 7 b7_w512
LZ4MT_AMD_BD_WARM_KIB=1024 run 7 b7_w1024
LZ4MT_AMD_BD_WARM_KIB=0 run 6 b6_w0
LZ4MT_AMD_BD_WARM_KIB=256 run 6 b6_w256
LZ4MT_AMD_BD_WARM_KIB=512 run 6 b6_w512
for f in $out/*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['compress_GiBps'], d['roofline']['kernel_ms'])"; done
for f in $out/*.err; do echo $f $(grep "encode\]" $f | tail -1); done
