# output staging ring (OB) in k_encode: encoder parity tests, then the headline bench and kstats
set -euo pipefail
out=gpurun_out/r02ao
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py tests/test_gpu_configs.py -m gpu > $out/tests.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $out/bench.json 2>$out/bench.err
timeout -k 10 300 python3 tools/kstats.py 8 7 > $out/kstats.txt 2>&1
