#!/bin/bash
# PMC passes on k_encode (each counter group in its own rocprofv3 run; no tracing domains).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); TAG=${TAG:-r01}
mkdir -p gpurun_out/pmc_${TAG}
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 2 --warmup 0 --no-cpu-baseline ${BENCH_ARGS}"
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_${TAG}/p$i" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_${TAG}/p$i.log" 2>&1 || exit $?
done
