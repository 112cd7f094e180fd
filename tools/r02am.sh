# chained -BD rounds: parity (test_gpu_bd.py) then 8 GiB B4 / B5 benches with stats
set -euo pipefail
out=gpurun_out/r02am
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bd.py tests/test_gpu_bd_hc.py > $out/tests.log 2>&1
export LZ4MT_AMD_BD_STATS=1
for b in 4 5; do
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --block-id $b --block-dependent --no-cpu-baseline > $out/bd$b.json 2>$out/bd$b.err
done
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --gib 1 --block-id 4 --block-dependent --no-cpu-baseline > $out/bd4_1g.json 2>$out/bd4_1g.err
