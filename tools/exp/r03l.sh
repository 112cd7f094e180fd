# kernel-trace stats of tools/ktime.py for every exp_libs/*.so (kernel times per variant)
set -euo pipefail
export TMPDIR=/tmp
for f in exp_libs/*.so; do
  nm=$(basename $f .so)
  LZ4MT_AMD_LIB=$f timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/$TAG/$nm -o t -- \
      python3 tools/ktime.py > gpurun_out/$TAG/$nm.txt 2>&1
  grep -v amdgpu gpurun_out/$TAG/$nm.txt
done
