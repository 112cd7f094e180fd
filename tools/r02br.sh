# HC two-link walk: A/B via LZ4MT_AMD_HC_LINK2, HC parity tests, short random campaign
set -euo pipefail
out=gpurun_out/r02br
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
  LZ4MT_AMD_HC_LINK2=0 timeout -k 10 200 python3 -u tools/hctime.py 2>&1 | grep -v amdgpu | sed 's/^/link2=0 /' >> $out/ab.txt
  timeout -k 10 200 python3 -u tools/hctime.py 2>&1 | grep -v amdgpu | sed 's/^/link2=1 /' >> $out/ab.txt
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_hc.py tests/test_gpu_bd_hc.py -m gpu > $out/tests.log 2>&1
timeout -k 10 200 python3 -u tools/fuzz_campaign.py 150 31 > $out/fuzz.txt 2>&1
