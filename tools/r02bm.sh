#!/bin/bash
# k_compact grid: 8192 blocks (default, 2 chunks per wave on C1) vs 1536 (one block per
# resident slot), 3072 and 16384 (one chunk per wave): interleaved A/B on C1 / C3 / C4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_ARGS="--no-memo-off-run --no-pipelined-run" timeout -k 10 900 bash tools/ab2.sh 1 3 4
