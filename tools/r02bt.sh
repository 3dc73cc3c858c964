#!/bin/bash
# k_encode under __launch_bounds__(64, 6) (80 VGPRs, 6 spill instructions; LDS then allows
# 21 one-wave blocks per CU) vs the default 5 (96 VGPRs, 20 blocks): C1 / C5 / C4, --verify
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TKZ_DEBUG=1 BENCH_ARGS="--no-memo-off-run --no-pipelined-run --verify" timeout -k 10 700 bash tools/ab2.sh 1 5 4 || exit $?
grep -h "blocks/CU" gpurun_out/ab2/*.err | sort | uniq -c
