# final refresh on the session's last encoder: profiles (kernel trace + FETCH/WRITE), headline bench with CPU
# baseline, block-size sweep, HC9, -BD B7, 32 GiB decompress-only, full GPU suite
set -euo pipefail
out=gpurun_out/r02bh
mkdir -p $out
export TMPDIR=/tmp
bash tools/prof.sh r02f > $out/prof.log 2>&1
timeout -k 10 400 python3 bench.py > $out/bench.json 2>$out/bench.err
for b in 4 5 6; do
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --block-id $b --no-cpu-baseline > $out/sweep_b$b.json 2>$out/sweep_b$b.err
done
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --level 9 --no-cpu-baseline > $out/hc9.json 2>$out/hc9.err
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --block-dependent --no-cpu-baseline > $out/bd7.json 2>$out/bd7.err
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --gib 32 --decompress-only --no-cpu-baseline > $out/dec32.json 2>$out/dec32.err
timeout -k 10 1100 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests -m gpu > $out/tests.log 2>&1
