# (round-4 scratch) A/B + full parity of the split-table exchange build
bash tools/gpu_round.sh r04xsp abbid && \
BID=5 LZ4MT_AMD_ENC=p17 bash tools/ab.sh > gpurun_out/r04xsp/ab_b5_p17.txt 2>&1; cat gpurun_out/r04xsp/ab_b5_p17.txt; \
LZ4MT_AMD_LIB=exp_libs/xsp.so timeout -k 10 1000 python3 -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests > gpurun_out/r04xsp/parity.log 2>&1; tail -3 gpurun_out/r04xsp/parity.log
