#!/bin/bash
# chunk size A/B (max chunk 8 KiB default vs 4 / 2 KiB): k_encode tail vs per-chunk costs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in ch12 ch11; do
  TKZ_LIB=$PWD/tokenizer-zig_amd/build/$lib.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bench or stream or golden" > gpurun_out/pytest_r02ad.log 2>&1 || { tail -30 gpurun_out/pytest_r02ad.log; exit 1; }
  tail -1 gpurun_out/pytest_r02ad.log
done
BENCH_ARGS="--no-memo-off-run" timeout -k 10 900 bash tools/ab2.sh 1 2 3 4 5
