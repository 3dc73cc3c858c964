#!/bin/bash
# Quick GPU check: parity tests, then bench (no CPU baseline) for the given configs.
# usage: TAG=x [SKIP_TESTS=1] bash tools/quick.sh [configs...]   (default: 1 2 3 4)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-q}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
  tail -1 gpurun_out/pytest_${TAG}.log
fi
[ $# -eq 0 ] && set -- 1 2 3 4
for c in "$@"; do
  timeout -k 10 300 python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --primary-only ${BENCH_ARGS} > gpurun_out/q_${TAG}_c$c.json 2> gpurun_out/q_${TAG}_c$c.err || { tail -20 gpurun_out/q_${TAG}_c$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/q_${TAG}_c$c.json'));k=d['roofline']['kernels'];print('C$c', round(d['value']/1e3,1), 'GB/s', d['ms_per_step'], 'ms/step', 'k_encode', k['k_encode']['avg_launch_ms'], k['other_ms'], 'verified', d['verified'] and d['verified']['sample_match'])"
done
