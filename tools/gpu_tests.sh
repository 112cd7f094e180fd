#!/bin/bash
# GPU parity tests only: tools/gpu_tests.sh <tag> [test files or -k expr...]
set -euo pipefail
tag=${1:-r02}; shift || true
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "$@" > "$out/pytest.log" 2>&1
tail -3 "$out/pytest.log"
