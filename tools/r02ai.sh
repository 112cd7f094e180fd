# full GPU suite + HC-BD benches (B7 split path, B4 segment path) + HC9 with CPU baseline
set -euo pipefail
out=gpurun_out/r02ai
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $out/tests.log 2>&1
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --block-dependent --level 9 > $out/bdhc7.json 2>$out/bdhc7.err
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --block-id 4 --block-dependent --level 9 --no-cpu-baseline > $out/bdhc4.json 2>$out/bdhc4.err
timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --level 9 > $out/hc9.json 2>$out/hc9.err
