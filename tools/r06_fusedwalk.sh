#!/bin/bash
# round 6: the frame walk fused into the decode (k_decode_walk) -- the
# diagnostic at every block size, the GPU parity file with every decode forced
# through it, then configs[2] (32 GiB decompress-only) and configs[1] with the
# separate serial walk vs fused
set -uo pipefail
out=gpurun_out/r06ac
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 120 python3 -u tools/walk_diag.py > "$out/diag.txt" 2>&1 || { tail -20 "$out/diag.txt"; exit 1; }
grep returned "$out/diag.txt"
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
