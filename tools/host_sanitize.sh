#!/bin/bash
# Host-code AddressSanitizer + UndefinedBehaviorSanitizer run of the CPU test
# suite's library paths (the host frame engine with CPU codecs, the I/O
# bindings, result tables, the gloo multi-process paths).  Device code is
# built as usual: every -fsanitize= sits behind -Xarch_host.  CPU only (no GPU
# run uses this build).  usage: bash tools/host_sanitize.sh [pytest args]
set -e
cd "$(dirname "$0")/.."
mkdir -p exp_libs
make -s clean >/dev/null
make -s -j8 EXTRA="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer -Xarch_host -shared-libsan" lz4mt_amd/liblz4mt_amd.so
cp lz4mt_amd/liblz4mt_amd.so exp_libs/asan.so
make -s clean >/dev/null
make -s -j8
ASANLIB=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
rm -f /tmp/lz4mt_asan.* /tmp/lz4mt_ubsan.*
LD_PRELOAD=$ASANLIB ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:log_path=/tmp/lz4mt_asan \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1:log_path=/tmp/lz4mt_ubsan \
LZ4MT_AMD_LIB=exp_libs/asan.so LZ4MT_AMD_LIB_OLDER=1 \
    python -m pytest tests/test_abi.py tests/test_dist.py -x -q -m "not gpu" "$@"
if ls /tmp/lz4mt_asan.* /tmp/lz4mt_ubsan.* >/dev/null 2>&1; then
    head -20 /tmp/lz4mt_asan.* /tmp/lz4mt_ubsan.* 2>/dev/null
    exit 1
fi
echo "no sanitizer reports"
