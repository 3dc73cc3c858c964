#!/bin/bash
# k_compact grid cap 65536 (default now) vs 8192: interleaved A/B on C1 / C3 / C4, then the
# full round run (smoke, GPU tests, bench lines, rocprof) and the PMC passes at this tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_ARGS="--no-memo-off-run --no-pipelined-run" timeout -k 10 600 bash tools/ab2.sh 1 3 4 > gpurun_out/r02bn_ab.txt 2>&1 || exit $?
for f in gpurun_out/ab2/c*_*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f', d['roofline']['k_compact']['ms'])"; done >> gpurun_out/r02bn_ab.txt
TAG=r02bn bash tools/gpu_r02.sh && TAG=r02bn bash tools/pmc_r02.sh
