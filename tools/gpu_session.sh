#!/bin/bash
# One GPU session: smoke -> GPU tests -> the default bench line -> rocprofv3 kernel trace of
# the primary region -> PMC passes over it (tools/pmc.sh). Each step has its own time limit;
# steps are chained (stop at the first failure).
#   usage: TAG=r03x [PYTEST_ARGS=...] [SKIP_TESTS=1] [SKIP_PMC=1] bash tools/gpu_session.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); TAG=${TAG:-r03}
D=gpurun_out/$TAG
mkdir -p $D
PRIMARY="--steps 5 --warmup 1 --primary-only --no-memo-off-run --no-pipelined-run --no-cpu-baseline --no-verify"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
    > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
  tail -1 $D/pytest.log
fi
timeout -k 10 900 python3 bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$D/trace" -o run --output-format csv -- \
  python3 "$R/bench.py" $PRIMARY > "$R/$D/trace.log" 2>&1 || { tail -20 "$R/$D/trace.log"; exit 1; }
cd "$R"
# the trace's per-kernel summary, stamped with the kernel-source hash (bench.py cites the
# committed profiles/<tag>_kernel_trace_summary.txt whose hash equals its build's)
{ echo "# src_hash $(python3 -c 'import bench; print(bench.kernel_src_hash())') (tools/trace_summary.py over $D/trace)";
  python3 tools/trace_summary.py "$(find $D/trace -name '*kernel_trace.csv' | head -1)"; } > $D/kernel_trace_summary.txt || exit 1
if [ -z "$SKIP_PMC" ]; then
  bash tools/pmc.sh $TAG python3 "$R/bench.py" --steps 2 --warmup 0 --primary-only --no-memo-off-run \
    --no-pipelined-run --no-cpu-baseline --no-verify || exit 1
fi
echo "session $TAG done"
