#!/bin/bash
# Compiler scheduling variants of the whole library (max-ilp, max-memory-clause, AMDGPU
# RP trackers, no loop alignment) vs the default build: interleaved A/B on C1 / C4 / C5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_ARGS="--no-memo-off-run" timeout -k 10 900 bash tools/ab2.sh 1 4 5
