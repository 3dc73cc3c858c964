#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TKZ_LIB=$PWD/tokenizer-zig_amd/build/wsync.so timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_hf_crosscheck.py tests/test_gpu_subbatch.py -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_subbatch.py::test_c4_shard_8M > gpurun_out/pytest_r02k.log 2>&1 || { tail -30 gpurun_out/pytest_r02k.log; exit 1; }
tail -1 gpurun_out/pytest_r02k.log
TKZ_LIB=$PWD/tools/wsync_phases.so timeout -k 10 120 python3 tools/phases.py 1 > gpurun_out/phases_wsync_c1.txt 2>&1 &&
BENCH_ARGS="--no-memo-off-run" timeout -k 10 600 bash tools/ab2.sh 1 3 4
