#!/bin/bash
# deferred-word dedup forced on for every BPE vocab (ddon) vs auto (multi-byte vocabs only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_ARGS="--no-memo-off-run" timeout -k 10 900 bash tools/ab2.sh 5 1 4
for f in gpurun_out/ab2/*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f'.split('/')[-1], d['roofline']['k_compact']['ms'], d['roofline']['other_kernels_ms'])"; done
