#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bench_configs or golden or edge" > gpurun_out/pytest_r02l.log 2>&1 || { tail -30 gpurun_out/pytest_r02l.log; exit 1; }
tail -1 gpurun_out/pytest_r02l.log
BENCH_ARGS="--no-memo-off-run" timeout -k 10 600 bash tools/ab2.sh 1 4
