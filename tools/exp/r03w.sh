# final-build validation: the whole GPU suite, then a time-boxed random differential campaign (seed 7)
set -euo pipefail
bash tools/gpu_round.sh r03w tests
timeout -k 10 420 python3 -u tools/fuzz_campaign.py 300 7 > gpurun_out/r03w/fuzz.txt 2>&1
tail -5 gpurun_out/r03w/fuzz.txt
