# K=32 count words by default: full GPU suite, profiles (kernel trace + FETCH/WRITE passes), bench with CPU baseline
set -euo pipefail
out=gpurun_out/r02ar
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $out/tests.log 2>&1
bash tools/prof.sh r02c > $out/prof.log 2>&1
timeout -k 10 400 python3 bench.py > $out/bench.json 2>$out/bench.err
