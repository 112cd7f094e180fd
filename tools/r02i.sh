set -euo pipefail
mkdir -p gpurun_out/r02i
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_bd.py -k "long_chains or golden_frames" > gpurun_out/r02i/pytest.log 2>&1
tail -2 gpurun_out/r02i/pytest.log
timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --gib 1 --block-dependent --no-cpu-baseline > gpurun_out/r02i/bench_bd.json 2>&1
timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --gib 1 --block-dependent --block-id 4 --no-cpu-baseline > gpurun_out/r02i/bench_bd4.json 2>&1
for f in gpurun_out/r02i/bench_*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['compress_GiBps'], d['decompress_GiBps'], d['ratio'], d['roofline']['kernel_ms'] if d['roofline'] else None)"; done
