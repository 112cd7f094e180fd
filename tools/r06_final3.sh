#!/bin/bash
# round 6, final build (SIMD-mate priority, fused walk for multi-generation frames, TRIM encoder,
# copy split 512 / 256 KiB): the GPU suite, smoke, the driver-shape bench, its kernel trace, the
# SQ / FETCH_SIZE passes, the end-to-end memory path
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06af
timeout -k 10 240 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > gpurun_out/r06af/smoke.txt 2>&1 || { tail -20 gpurun_out/r06af/smoke.txt; exit 1; }
bash tools/gpu_round.sh r06af tests bench trace sweep fuzz
