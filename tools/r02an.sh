# re-entry check: full GPU suite, headline bench with CPU baseline, kernel stats
set -euo pipefail
out=gpurun_out/r02an
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $out/tests.log 2>&1
timeout -k 10 400 python3 bench.py > $out/bench.json 2>$out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $out/trace -o trace -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $out/bench_prof.log 2>&1
timeout -k 10 300 python3 tools/kstats.py 8 7 > $out/kstats.txt 2>&1
