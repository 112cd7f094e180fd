set -euo pipefail
out=gpurun_out/r02m
mkdir -p $out
export TMPDIR=/tmp
df -h /dev/shm /tmp > $out/df.txt 2>&1 || true
timeout -k 10 600 python3 -u tools/e2e.py 8 7 --file /dev/shm > $out/e2e_file.txt 2>&1
timeout -k 10 600 python3 -u tools/e2e.py 8 7 > $out/e2e_mem.txt 2>&1
cat $out/df.txt $out/e2e_file.txt $out/e2e_mem.txt | grep -v amdgpu
