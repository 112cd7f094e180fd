# random differential campaign with -BD cases (liblz4 1.9.3 stream API as the reference's call sequence)
set -euo pipefail
out=gpurun_out/r02bo
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/fuzz_campaign.py 240 21 > $out/fuzz_s21.txt 2>&1
timeout -k 10 300 python3 -u tools/fuzz_campaign.py 240 22 > $out/fuzz_s22.txt 2>&1
