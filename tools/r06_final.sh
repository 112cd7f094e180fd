#!/bin/bash
# round 6, final build (TRIM encoder default, copy-pool fix and 512 / 256 KiB
# split): the GPU suite, smoke, the driver-shape bench, its kernel trace, the
# SQ / FETCH_SIZE passes, the end-to-end memory path
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06o
timeout -k 10 240 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > gpurun_out/r06o/smoke.txt 2>&1 || { tail -20 gpurun_out/r06o/smoke.txt; exit 1; }
bash tools/gpu_round.sh r06o tests bench trace sq pmc e2ems
