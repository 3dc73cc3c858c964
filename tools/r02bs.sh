#!/bin/bash
# k_compact tokens per lane per emission round (TKZ_COMPACT_MINB 1 default (6 waves/SIMD at 80 VGPRs) vs 7 (72 VGPRs, 6 spills)) with the
# one-chunk-per-wave grid: interleaved A/B on C1 / C3 / C4 (k_compact ms from the lines)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_ARGS="--no-memo-off-run --no-pipelined-run" timeout -k 10 600 bash tools/ab2.sh 1 3 4 || exit $?
for f in gpurun_out/ab2/c*_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', d['roofline']['k_compact']['ms'])"; done
