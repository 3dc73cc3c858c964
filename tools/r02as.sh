#!/bin/bash
# split scan/resolve with LDS-staged entries: parity, A/B vs fused, per-kernel trace of C1
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out/as
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not stream" > gpurun_out/pytest_r02as.log 2>&1 || { tail -40 gpurun_out/pytest_r02as.log; exit 1; }
tail -1 gpurun_out/pytest_r02as.log
BENCH_ARGS="--no-memo-off-run" timeout -k 10 900 bash tools/ab2.sh 1 4 5
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/as/c1" -o run --output-format csv -- python3 "$R/bench.py" --config 1 --steps 10 --warmup 2 --no-cpu-baseline --no-memo-off-run > "$R/gpurun_out/as/c1.json" 2> "$R/gpurun_out/as/c1.err") || exit 1
python3 tools/trace_summary.py $(find gpurun_out/as/c1 -name '*kernel_trace.csv' | head -1) | head -8
