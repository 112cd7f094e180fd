#!/bin/bash
# round 6: configs[2] (32 GiB decompress-only) and configs[1] on the default
# build (the fused walk chosen for frames of more than one decode generation)
set -uo pipefail
out=gpurun_out/r06ag
mkdir -p "$out"
export TMPDIR=/tmp
for pass in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --gib 32 --decompress-only --steps 3 --warmup 1 > "$out/dec32_$pass.json" 2> "$out/dec32_$pass.err" || exit 1
  echo "dec32 pass $pass: $(grep -o '"ms_per_step": [0-9.]*' "$out/dec32_$pass.json") $(grep -o '"value": [0-9.]*' "$out/dec32_$pass.json" | head -1)"
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > "$out/b7.json" 2> "$out/b7.err" || exit 1
echo "b7: $(grep -o '"value": [0-9.]*\|"decompress_GiBps": [0-9.]*' "$out/b7.json" | head -2 | tr '\n' ' ')"
timeout -k 10 400 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_configs.py -k "32gib or dec" > "$out/configs.txt" 2>&1; tail -1 "$out/configs.txt"
