#!/bin/bash
# k_dedup_copy with batched loads: parity (dedup-relevant GPU tests), then A/B on C2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_subbatch.py -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_subbatch.py::test_c4_shard_8M > gpurun_out/pytest_r02q.log 2>&1 || { tail -40 gpurun_out/pytest_r02q.log; exit 1; }
tail -1 gpurun_out/pytest_r02q.log
BENCH_ARGS="--no-memo-off-run" timeout -k 10 600 bash tools/ab2.sh 2
