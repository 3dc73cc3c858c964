#!/bin/bash
# k_dedup_copy with 2 (default) / 1 / 4 repeats per lane and iteration: parity (dedup tests), then C2 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dedup or parity or subbatch" > gpurun_out/pytest_r02be.log 2>&1 || { tail -40 gpurun_out/pytest_r02be.log; exit 1; }
tail -1 gpurun_out/pytest_r02be.log
BENCH_ARGS="--no-memo-off-run" timeout -k 10 900 bash tools/ab2.sh 2
