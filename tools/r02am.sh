#!/bin/bash
# per-kernel breakdown of the deferred phase on C2 / C4 / C5 (kernel trace)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out/r02am
for c in 2 4 5; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r02am/c$c" -o run --output-format csv -- python3 "$R/bench.py" --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-memo-off-run > "$R/gpurun_out/r02am/c$c.json" 2> "$R/gpurun_out/r02am/c$c.err") || exit 1
  f=$(find gpurun_out/r02am/c$c -name '*kernel_trace.csv' | head -1)
  echo "== C$c"; python3 tools/trace_summary.py "$f"
done
