# more seeds of the random differential campaign
set -euo pipefail
out=gpurun_out/r02bs
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 330 python3 -u tools/fuzz_campaign.py 270 41 > $out/fuzz_s41.txt 2>&1
timeout -k 10 330 python3 -u tools/fuzz_campaign.py 270 42 > $out/fuzz_s42.txt 2>&1
