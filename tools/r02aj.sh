# 3-byte-table encoder (k_encode_p17) A/B: parity with LZ4MT_AMD_ENC=p17, then B5/B6/B7 benches both ways
set -euo pipefail
out=gpurun_out/r02aj
mkdir -p $out
export TMPDIR=/tmp
LZ4MT_AMD_ENC=p17 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py tests/test_gpu_configs.py > $out/tests_p17.log 2>&1
for b in 7 6 5; do
for e in base p17; do
LZ4MT_AMD_ENC=$e timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --block-id $b --no-cpu-baseline > $out/b${b}_$e.json 2>$out/b${b}_$e.err
done
done
