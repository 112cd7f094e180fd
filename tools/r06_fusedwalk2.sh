#!/bin/bash
# round 6: fused walk with 8 decoders per CU + the walker: parity (GPU file,
# fused forced) and configs[2] / configs[1], serial vs fused, two passes
set -uo pipefail
out=gpurun_out/r06ae
mkdir -p "$out"
export TMPDIR=/tmp
LZ4MT_AMD_WALK=fused timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py > "$out/test_gpu_fused.txt" 2>&1 || { tail -30 "$out/test_gpu_fused.txt"; exit 1; }
tail -1 "$out/test_gpu_fused.txt"
for pass in 1 2; do
  for w in serial fused; do
    LZ4MT_AMD_WALK=$w timeout -k 10 300 python3 bench.py --no-cpu-baseline --gib 32 --decompress-only --steps 3 --warmup 1 > "$out/dec32_${w}_$pass.json" 2> "$out/dec32_${w}_$pass.err" || exit 1
    echo "dec32 $w pass $pass: $(grep -o '"ms_per_step": [0-9.]*' "$out/dec32_${w}_$pass.json") $(grep -o '"value": [0-9.]*' "$out/dec32_${w}_$pass.json" | head -1)"
    LZ4MT_AMD_WALK=$w timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > "$out/b7_${w}_$pass.json" 2> "$out/b7_${w}_$pass.err" || exit 1
    echo "b7 $w pass $pass: $(grep -o '"value": [0-9.]*\|"decompress_GiBps": [0-9.]*' "$out/b7_${w}_$pass.json" | head -2 | tr '\n' ' ')"
  done
done
