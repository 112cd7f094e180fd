# time-boxed random differential campaign: device frames vs the oracle, two seeds
set -euo pipefail
out=gpurun_out/r02bn
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 330 python3 -u tools/fuzz_campaign.py 270 11 > $out/fuzz_s11.txt 2>&1
timeout -k 10 330 python3 -u tools/fuzz_campaign.py 270 12 > $out/fuzz_s12.txt 2>&1
