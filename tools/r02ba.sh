#!/bin/bash
# per-wave LDS cache of short memo misses: parity, then A/B vs TKZ_MCACHE=0
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not stream" > gpurun_out/pytest_r02ba.log 2>&1 || { tail -40 gpurun_out/pytest_r02ba.log; exit 1; }
tail -1 gpurun_out/pytest_r02ba.log
BENCH_ARGS="--no-memo-off-run" timeout -k 10 900 bash tools/ab2.sh 5 1 4 2
