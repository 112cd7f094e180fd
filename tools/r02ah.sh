# HC: parity (HC + HC-BD GPU tests) then level 9 / 3 at 8 GiB B7 for several stream lengths
set -euo pipefail
out=gpurun_out/r02ah
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hc.py tests/test_gpu_bd_hc.py > $out/tests.log 2>&1
export LZ4MT_AMD_HC_STATS=1
for sub in 256 128 512; do
LZ4MT_AMD_HC_SUB_KIB=$sub timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --level 9 --no-cpu-baseline > $out/hc9_s$sub.json 2>$out/hc9_s$sub.err
done
LZ4MT_AMD_HC_SUB_KIB=256 timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --level 3 --no-cpu-baseline > $out/hc3_s256.json 2>$out/hc3_s256.err
LZ4MT_AMD_HC_SUB_KIB=256 timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --level 9 --block-id 6 --no-cpu-baseline > $out/hc9b6_s256.json 2>$out/hc9b6_s256.err
cd /tmp && LZ4MT_AMD_HC_SUB_KIB=256 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --level 9 --no-cpu-baseline > $GRAFT_REPO_ROOT/$out/prof.log 2>&1
