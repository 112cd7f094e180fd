# final state of the session's encoder changes: full GPU suite, profiles (kernel trace + FETCH/WRITE), bench
set -euo pipefail
out=gpurun_out/r02az
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $out/tests.log 2>&1
bash tools/prof.sh r02e > $out/prof.log 2>&1
timeout -k 10 400 python3 bench.py > $out/bench.json 2>$out/bench.err
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --block-id 6 --no-cpu-baseline > $out/sweep_b6.json 2>$out/sweep_b6.err
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --block-id 5 --no-cpu-baseline > $out/sweep_b5.json 2>$out/sweep_b5.err
