#!/bin/bash
# A/B kernel timing of every exp_libs/*.so (run on the GPU box): tools/ab.sh > gpurun_out/ab.txt
for f in exp_libs/*.so; do
  LZ4MT_AMD_LIB_OLDER=1 LZ4MT_AMD_LIB=$f timeout -k 10 120 python3 -u tools/ktime.py 2>&1 | grep -v amdgpu || exit 1
done
