#!/bin/bash
# k_compact software pipeline (next group prefetched): parity, then A/B vs TKZ_COMPACT_PF=0
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not stream" > gpurun_out/pytest_r02ax.log 2>&1 || { tail -40 gpurun_out/pytest_r02ax.log; exit 1; }
tail -1 gpurun_out/pytest_r02ax.log
BENCH_ARGS="--no-memo-off-run" timeout -k 10 900 bash tools/ab2.sh 1 4 3 5
