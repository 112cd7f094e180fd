#!/bin/bash
# round 6, final build (SIMD-mate priority in the encoder and decoder, TRIM encoder,
# copy split 512 / 256 KiB): the GPU suite, smoke, the driver-shape bench, its kernel trace, the
# SQ / FETCH_SIZE passes, the end-to-end memory path
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06y
timeout -k 10 240 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > gpurun_out/r06y/smoke.txt 2>&1 || { tail -20 gpurun_out/r06y/smoke.txt; exit 1; }
bash tools/gpu_round.sh r06y tests bench trace sq pmc pmc32 e2ems sweep
