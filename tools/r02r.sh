set -euo pipefail
out=gpurun_out/r02v
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --level 9 > $out/bench_hc9.json 2>$out/hc9.err
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --level 3 > $out/bench_hc3.json 2>$out/hc3.err
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --gib 1 --block-dependent > $out/bench_bd7.json 2>$out/bd7.err
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --gib 1 --block-dependent --block-id 4 > $out/bench_bd4.json 2>$out/bd4.err
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --stream-checksum > $out/bench_sck.json 2>$out/sck.err
timeout -k 10 600 python3 bench.py > $out/bench_default.json 2>$out/default.err
for f in $out/bench_*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['cpu_baseline'] or {}; print('$f', d['value'], d['compress_GiBps'], d['decompress_GiBps'], d['ratio'], d['roofline']['kernel'], d['roofline']['kernel_ms'], '| cpu', c.get('value'), c.get('compress_GiBps'), c.get('decompress_GiBps'), c.get('cores'))"; done
