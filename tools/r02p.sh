#!/bin/bash
# Kernel traces of C2 (dedup path) and C5 (disjoint lexicon) bench commands.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out/r02p
cd /tmp && export TMPDIR=/tmp
for c in 2 5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02p/c$c" -o run --output-format csv -- python3 "$R/bench.py" --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-memo-off-run > "$R/gpurun_out/r02p/c$c.log" 2>&1 || exit $?
done
