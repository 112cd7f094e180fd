# optimal parser on the split path: HC parity tests, then 8 GiB benches at levels 10 / 12
set -euo pipefail
out=gpurun_out/r02bd
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_hc.py -m gpu > $out/tests.log 2>&1
LZ4MT_AMD_HC_STATS=1 timeout -k 10 400 python3 bench.py --gib 8 --steps 1 --warmup 1 --level 10 > $out/hc10.json 2>$out/hc10.err
timeout -k 10 500 python3 bench.py --gib 8 --steps 1 --warmup 1 --level 12 > $out/hc12.json 2>$out/hc12.err
