# optimal parser with the price array in LDS: HC parity tests, then 8 GiB benches at levels 10 / 12
set -euo pipefail
out=gpurun_out/r02bi
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_hc.py -m gpu > $out/tests.log 2>&1
timeout -k 10 300 python3 bench.py --gib 8 --steps 1 --warmup 1 --level 10 --no-cpu-baseline > $out/hc10.json 2>$out/hc10.err
timeout -k 10 300 python3 bench.py --gib 8 --steps 1 --warmup 1 --level 12 --no-cpu-baseline > $out/hc12.json 2>$out/hc12.err
