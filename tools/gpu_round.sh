#!/bin/bash
# One GPU session: smoke -> GPU parity tests -> bench (memo on/off, all configs) -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; steps are chained with && (stop at the first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 1200 python3 -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 600 python3 bench.py --steps 5 --warmup 1 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err &&
timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-memo --no-cpu-baseline > gpurun_out/bench_${TAG}_nomemo.json 2>> gpurun_out/bench_${TAG}.err &&
for c in 2 3 4; do timeout -k 10 300 python3 bench.py --config $c --steps 5 --warmup 1 --cpu-sample-docs 200000 --cpu-min-seconds 3 > gpurun_out/bench_${TAG}_c$c.json 2>> gpurun_out/bench_${TAG}.err || exit $?; done &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/prof_${TAG}.log" 2>&1
