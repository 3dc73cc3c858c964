#!/bin/bash
# scratch array bases rematerialised from base/tb at each use (remat) vs hoisted + spilled (default)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_ARGS="--no-memo-off-run" timeout -k 10 900 bash tools/ab2.sh 1 4 5 2
