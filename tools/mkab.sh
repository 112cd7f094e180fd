#!/bin/bash
# Builds exp_libs/head.so (HEAD's kernels) and exp_libs/<name>.so (the working tree) for tools/ab.sh.
# usage: tools/mkab.sh <name> [extra hipcc flags for the working-tree build]
set -e
name=$1; shift || true
mkdir -p exp_libs; rm -f exp_libs/*.so
make -s clean >/dev/null; make -s -j8 EXTRA="$*" lz4mt_amd/liblz4mt_amd.so; cp lz4mt_amd/liblz4mt_amd.so exp_libs/$name.so
git stash -q; make -s clean >/dev/null; make -s -j8 lz4mt_amd/liblz4mt_amd.so; cp lz4mt_amd/liblz4mt_amd.so exp_libs/head.so; git stash pop -q
make -s clean >/dev/null; make -s -j8
ls exp_libs
