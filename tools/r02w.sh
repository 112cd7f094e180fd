set -euo pipefail
out=gpurun_out/r02w
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_hc.py > $out/pytest.log 2>&1
tail -1 $out/pytest.log
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --level 9 --no-cpu-baseline > $out/bench_hc9.json 2>$out/hc9.err
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --level 3 --no-cpu-baseline > $out/bench_hc3.json 2>$out/hc3.err
for f in $out/bench_*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['compress_GiBps'], d['decompress_GiBps'], d['ratio'], d['roofline']['kernel_ms'])"; done
