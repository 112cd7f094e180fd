set -euo pipefail
mkdir -p gpurun_out/r02g
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/ > gpurun_out/r02g/pytest.log 2>&1
tail -2 gpurun_out/r02g/pytest.log
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02g/bench_default.json 2>&1
timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --gib 1 --block-dependent --no-cpu-baseline > gpurun_out/r02g/bench_bd.json 2>&1
timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --gib 1 --block-dependent --block-id 4 --no-cpu-baseline > gpurun_out/r02g/bench_bd4.json 2>&1
for f in gpurun_out/r02g/bench_*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d.get('compress_GiBps'), d.get('decompress_GiBps'), d.get('ratio'), d['roofline'])"; done
