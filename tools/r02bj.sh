# XXH32 wave with 4 KiB chunks: frame/checksum GPU tests, then kernel-trace stats of the headline bench
set -euo pipefail
out=gpurun_out/r02bj
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py tests/test_gpu_configs.py -m gpu > $out/tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $out/trace -o trace -- \
    python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $out/bench.json 2>$out/bench.err
