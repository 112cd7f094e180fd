#!/bin/bash
# Builds compile-time variants of the working tree's library for tools/ab.sh:
#   tools/mkvariants.sh base= pf1=-DLZ4MT_PF=1 pf2=-DLZ4MT_PF=2
# -> exp_libs/base.so, exp_libs/pf1.so, ... (then the product library is rebuilt as is)
set -e
mkdir -p exp_libs; rm -f exp_libs/*.so
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  make -s clean >/dev/null; make -s -j8 EXTRA="$flags" lz4mt_amd/liblz4mt_amd.so
  cp lz4mt_amd/liblz4mt_amd.so exp_libs/$name.so
done
make -s clean >/dev/null; make -s -j8
ls -la exp_libs
