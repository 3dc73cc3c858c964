#!/bin/bash
# Kernel trace of whole-doc pretoken configs (the segmented path): for each config in
# $CFGS, rocprofv3 --kernel-trace --stats over `bench.py --config C --primary-only`
# (2 timed steps), summarised per kernel and iteration by tools/trace_summary.py.
#   usage: TAG=r05d CFGS="8 9" bash tools/seg_trace.sh [extra bench.py args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); TAG=${TAG:-seg}
D=gpurun_out/$TAG
mkdir -p $D
for C in ${CFGS:-6 8 9}; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$D/trace_c$C" -o run \
    --output-format csv -- python3 "$R/bench.py" --config $C --steps 2 --warmup 1 --primary-only --no-memo-off-run \
    --no-pipelined-run --no-cpu-baseline --no-verify --no-host-e2e "$@" > "$R/$D/trace_c$C.log" 2>&1) \
    || { tail -20 "$R/$D/trace_c$C.log"; exit 1; }
  f=$(find "$R/$D/trace_c$C" -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_summary.py "$f" > "$D/summary_c$C.txt" && head -30 "$D/summary_c$C.txt"
done
