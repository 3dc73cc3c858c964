#!/bin/bash
# k_emit (lane-per-word emission, memo-slot references): GPU tests, then interleaved A/B
# against the previous HEAD build (build/head.so) and variants in build/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_subbatch.py::test_c4_shard_8M > gpurun_out/pytest_r02n.log 2>&1 || { tail -40 gpurun_out/pytest_r02n.log; exit 1; }
tail -1 gpurun_out/pytest_r02n.log
BENCH_ARGS="--no-memo-off-run" timeout -k 10 900 bash tools/ab2.sh 1 2 3 4 5
