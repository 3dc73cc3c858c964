#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/valu_mix > gpurun_out/valu_mix.jsonl 2>&1 &&
TKZ_LIB=$PWD/tokenizer-zig_amd/build/phases.so timeout -k 10 120 python3 tools/phases.py 1 > gpurun_out/phases_c1.txt 2>&1 &&
TKZ_LIB=$PWD/tokenizer-zig_amd/build/phases.so timeout -k 10 120 python3 tools/phases.py 5 > gpurun_out/phases_c5.txt 2>&1 &&
BENCH_ARGS="--no-memo-off-run" timeout -k 10 600 bash tools/ab2.sh 1
