#!/bin/bash
# Kernel traces of one config under several libraries (the in-tree libtkz.so and the variants
# in tokenizer-zig_amd/build/), summarised per kernel by tools/trace_summary.py.
#   usage: TAG=r06h CFG=6 bash tools/trace_ab.sh [extra bench.py args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); TAG=${TAG:-tab}; CFG=${CFG:-6}
D=gpurun_out/$TAG
mkdir -p $D
for lib in tokenizer-zig_amd/tkz/libtkz.so $(ls tokenizer-zig_amd/build/*.so 2>/dev/null); do
  n=$(basename $lib .so)
  (cd /tmp && export TMPDIR=/tmp && TKZ_LIB=$R/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    -d "$R/$D/trace_${n}_c$CFG" -o run --output-format csv -- python3 "$R/bench.py" --config $CFG --steps 2 --warmup 1 \
    --primary-only --no-memo-off-run --no-pipelined-run --no-cpu-baseline --no-verify --no-host-e2e "$@" \
    > "$R/$D/trace_${n}_c$CFG.log" 2>&1) || { tail -20 "$R/$D/trace_${n}_c$CFG.log"; exit 1; }
  f=$(find "$R/$D/trace_${n}_c$CFG" -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_summary.py "$f" > "$D/summary_${n}_c$CFG.txt" || exit 1
done
