#!/bin/bash
# CPU test suite (-m "not gpu") against AddressSanitizer + UBSan builds of the host code:
# libtkz (loader, JSON parser, tables, decode, pools), libtkzsynth and the C++ oracle.
# Runs in the build container (no GPU). usage: bash tools/asan_cpu_tests.sh [pytest args]
set -eo pipefail
cd "$(dirname "$0")/.."
make -s -C tokenizer-zig_amd asan
make -s -C oracle asan
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
export TKZ_LIB=$PWD/tokenizer-zig_amd/tkz/asan/libtkz.so
export TKZ_SYNTH_LIB=$PWD/tokenizer-zig_amd/tkz/asan/libtkzsynth.so
export TKZ_ORACLE_LIB=$PWD/oracle/build/asan/liboracle.so
# leaks: the Python interpreter itself is not leak-clean; UBSan findings abort the test
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD=$RT python3 -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
