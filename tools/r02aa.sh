set -euo pipefail
out=gpurun_out/r02aa
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_bd.py > $out/pytest.log 2>&1
tail -1 $out/pytest.log
export LZ4MT_AMD_BD_STATS=1
for bid in 7 6 5; do
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --gib 1 --block-dependent --block-id $bid --no-cpu-baseline > $out/bd$bid.json 2>$out/bd$bid.err
LZ4MT_AMD_BD_COLD=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --gib 1 --block-dependent --block-id $bid --no-cpu-baseline > $out/bd${bid}_cold.json 2>$out/bd${bid}_cold.err
done
timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --gib 8 --block-dependent --block-id 7 --no-cpu-baseline > $out/bd7_8g.json 2>$out/bd7_8g.err
for f in $out/bd*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['compress_GiBps'], d['decompress_GiBps'], d['roofline']['kernel_ms'])"; done
grep -h "encode\]" $out/bd7.err $out/bd6.err $out/bd5.err $out/bd7_8g.err | sort | uniq -c | head
