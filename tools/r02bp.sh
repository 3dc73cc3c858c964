#!/bin/bash
# deferred-phase grid (8 blocks per CU default vs 16 / 4) and k_chunk_count grid cap (8192
# default vs 65536): interleaved A/B on C1 / C2 / C5 / C4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_ARGS="--no-memo-off-run --no-pipelined-run" timeout -k 10 900 bash tools/ab2.sh 1 2 5 4
