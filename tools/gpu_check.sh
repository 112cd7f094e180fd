#!/bin/bash
# One GPU-box pass: parity tests, the 1-GPU bench line, the default-flag
# bench line.  Each step has its own time limit; the first failure ends it.
# usage: tools/gpu_check.sh <tag> [pytest -k expr]
set -euo pipefail
tag=${1:-r02}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
kexpr=${2:-}
if [ -n "$kexpr" ]; then
  timeout -k 10 900 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 \
      --timeout-method thread -k "$kexpr" > "$out/pytest.log" 2>&1
else
  timeout -k 10 900 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 \
      --timeout-method thread > "$out/pytest.log" 2>&1
fi
tail -3 "$out/pytest.log"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err"
cat "$out/bench.json"
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --stream-checksum --no-cpu-baseline > "$out/bench_sck.json" 2> "$out/bench_sck.err"
cat "$out/bench_sck.json"
