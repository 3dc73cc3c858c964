#!/bin/bash
# timing-only ablations of k_resolve (split build): a4 misses dropped, a5 memo without memory, a8 no key loads + misses dropped
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_ARGS="--no-memo-off-run" timeout -k 10 900 bash tools/ab2.sh 1 5
