#!/bin/bash
# register BPE: adjacent-pair probe after a one-merge round (PROBE3 3 default, 1, 0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not stream" > gpurun_out/pytest_r02ap.log 2>&1 || { tail -30 gpurun_out/pytest_r02ap.log; exit 1; }
tail -1 gpurun_out/pytest_r02ap.log


BENCH_ARGS="--no-memo-off-run" timeout -k 10 900 bash tools/ab2.sh 1 5 2 4
for f in gpurun_out/ab2/*_1.json; do python3 -c "import json;d=json.load(open('$f'));print('$f'.split('/')[-1], d.get('memo'))"; done
