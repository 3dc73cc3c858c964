#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_ARGS="--no-memo-off-run" timeout -k 10 600 bash tools/ab2.sh 1 5 > gpurun_out/ab2_r02c.txt 2>&1 &&
TAG=r02c timeout -k 10 900 bash tools/pmc_r02.sh
