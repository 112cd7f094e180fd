# FETCH_SIZE of k_encode with 63 / 32 / 16 forward-count words (8 GiB App. F, B7)
set -euo pipefail
out=gpurun_out/r02aq
mkdir -p $out
export TMPDIR=/tmp
for k in 63 32 16; do
  LZ4MT_AMD_LIB=exp_libs/k$k.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -T -f csv -d $out/fetch_k$k -o fetch -- python3 tools/kprof.py 8 > $out/fetch_k$k.log 2>&1
done
