#!/bin/bash
# runtime memo slots for short misses: parity, then A/B vs TKZ_MEMO_INS=0
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not stream" > gpurun_out/pytest_r02au.log 2>&1 || { tail -40 gpurun_out/pytest_r02au.log; exit 1; }
tail -1 gpurun_out/pytest_r02au.log
BENCH_ARGS="--no-memo-off-run" timeout -k 10 900 bash tools/ab2.sh 5 1 4
for f in gpurun_out/ab2/*_1.json; do python3 -c "import json;d=json.load(open(\"$f\"));print(\"$f\".split(\"/\")[-1], d.get(\"memo\"))"; done
