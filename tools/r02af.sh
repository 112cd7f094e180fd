# -BD at level 9 (the HC stream): bench B7 / B4 at 8 GiB + kernel stats
set -euo pipefail
out=gpurun_out/r02af
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --gib 8 --block-dependent --level 9 > $out/bdhc7.json 2>$out/bdhc7.err
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --gib 8 --block-id 4 --block-dependent --level 9 --no-cpu-baseline > $out/bdhc4.json 2>$out/bdhc4.err
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --gib 8 --block-id 4 --block-dependent --level 9 --no-cpu-baseline > $GRAFT_REPO_ROOT/$out/prof.log 2>&1
