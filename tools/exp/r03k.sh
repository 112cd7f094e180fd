set -euo pipefail
mkdir -p gpurun_out/r03k
export TMPDIR=/tmp
for k in 1 2; do for f in exp_nost/base.so exp_nost/nost.so; do
  LZ4MT_AMD_LIB=$f timeout -k 10 120 python3 -u tools/enc_only.py 2>&1 | grep -v amdgpu | tee -a gpurun_out/r03k/nost.txt
done; done
ABLIB=asm4 bash tools/gpu_round.sh r03k ab abtest
