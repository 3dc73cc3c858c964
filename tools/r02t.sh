#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in 1 3 4 5; do timeout -k 10 300 python3 tools/bench_streams.py $c 2 20 || exit $?; done
timeout -k 10 300 python3 tools/bench_streams.py 1 3 21
