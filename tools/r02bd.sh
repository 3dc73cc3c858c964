#!/bin/bash
# k_chunk_count with two groups' count loads in flight per iteration (default) vs one (cu1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"


BENCH_ARGS="--no-memo-off-run" timeout -k 10 900 bash tools/ab2.sh 1 4 5
