set -euo pipefail
out=gpurun_out/r02ae
mkdir -p $out
export TMPDIR=/tmp LZ4MT_AMD_BD_STATS=1
for w in 1024 1536 2048; do
LZ4MT_AMD_BD_WARM_KIB=$w timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --gib 8 --block-dependent --no-cpu-baseline > $out/w$w.json 2>$out/w$w.err
done
for f in $out/*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['compress_GiBps'], d['roofline']['kernel_ms'])"; done
for f in $out/*.err; do echo $f $(grep "encode\]" $f | tail -2); done
