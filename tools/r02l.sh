set -euo pipefail
out=gpurun_out/r02l
mkdir -p $out
export TMPDIR=/tmp
for bid in 6 7; do
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --block-id $bid --no-cpu-baseline > $out/base_b$bid.json 2>&1
timeout -k 10 300 python3 exp_occ/bench.py --steps 2 --warmup 1 --block-id $bid --no-cpu-baseline > $out/exp_b$bid.json 2>&1
done
for f in $out/*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['compress_GiBps'], d['ratio'], d['roofline']['kernel_ms'])"; done
