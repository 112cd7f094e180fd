# 4-wave k_hc_prev: HC + HC-BD parity, then HC9 B7 and -BD HC B4 benches
set -euo pipefail
out=gpurun_out/r02ak
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hc.py tests/test_gpu_bd_hc.py > $out/tests.log 2>&1
timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --level 9 --no-cpu-baseline > $out/hc9.json 2>$out/hc9.err
timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --level 3 --no-cpu-baseline > $out/hc3.json 2>$out/hc3.err
timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --block-id 4 --block-dependent --level 9 --no-cpu-baseline > $out/bdhc4.json 2>$out/bdhc4.err
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --level 9 --no-cpu-baseline > $GRAFT_REPO_ROOT/$out/prof.log 2>&1
