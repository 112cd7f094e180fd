set -euo pipefail
out=gpurun_out/r02p
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/kstats.py 8 7 > $out/kstats.txt 2>&1
grep -v amdgpu $out/kstats.txt
