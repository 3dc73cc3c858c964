#!/bin/bash
# GPU parity tests, then interleaved A/B timing (tools/ab2.sh) for the configs given.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || { tail -30 gpurun_out/pytest_ab.log; exit 1; }
tail -1 gpurun_out/pytest_ab.log
bash tools/ab2.sh "$@"
