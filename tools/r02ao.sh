#!/bin/bash
# k_dedup first-launch size 4096 / 16384 / 262144 vs 65536
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out


BENCH_ARGS="--no-memo-off-run" timeout -k 10 900 bash tools/ab2.sh 2
for f in gpurun_out/ab2/*_1.json; do python3 -c "import json;d=json.load(open('$f'));print('$f'.split('/')[-1], d.get('memo'))"; done
