#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in tokenizer-zig_amd/tkz/libtkz.so tokenizer-zig_amd/build/nopf.so; do
TKZ_LIB=$PWD/$L timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_hf_crosscheck.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bench_configs or golden or edge or random or hf" > gpurun_out/pytest_r02h.log 2>&1 || { tail -30 gpurun_out/pytest_r02h.log; exit 1; }
tail -1 gpurun_out/pytest_r02h.log
done
BENCH_ARGS="--no-memo-off-run" timeout -k 10 600 bash tools/ab2.sh 1 3 4
