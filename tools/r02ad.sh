set -euo pipefail
out=gpurun_out/r02ad
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_bd.py > $out/pytest_bd.log 2>&1
tail -1 $out/pytest_bd.log
timeout -k 10 600 python3 -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu.py -k "compress or frames_golden or known_answers" > $out/pytest_enc.log 2>&1
tail -1 $out/pytest_enc.log
export LZ4MT_AMD_BD_STATS=1
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --gib 1 --block-dependent --no-cpu-baseline > $out/bd7.json 2>$out/bd7.err
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --gib 1 --block-dependent --block-id 4 --no-cpu-baseline > $out/bd4.json 2>$out/bd4.err
timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --gib 8 --block-dependent --no-cpu-baseline > $out/bd7_8g.json 2>$out/bd7_8g.err
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/default.json 2>$out/default.err
for f in $out/*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['compress_GiBps'], d['decompress_GiBps'], d['roofline']['kernel_ms'])"; done
for f in $out/bd*.err; do echo $f $(grep "encode\]" $f | tail -1); done
