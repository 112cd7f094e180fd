set -euo pipefail
out=gpurun_out/r02x
mkdir -p $out
export TMPDIR=/tmp
for f in exp_libs/*.so; do
  LZ4MT_AMD_LIB=$f timeout -k 10 300 python3 -u tools/hctime.py 2>&1 | grep -v amdgpu
done > $out/ab.txt
cat $out/ab.txt
