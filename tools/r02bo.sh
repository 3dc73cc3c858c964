#!/bin/bash
# k_compact grid cap 65536 (default) vs 16384 vs 8192 on the C4 8M-doc shard (2 passes of
# 3.9 GB) and on C4 / C1 at 1M docs, with --verify (first 100k docs vs the oracle)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_ARGS="--no-memo-off-run --no-pipelined-run --verify --docs 8000000" timeout -k 10 700 bash tools/ab2.sh 4 || exit $?
for f in gpurun_out/ab2/c4_*.json; do python3 -c "import json;d=json.load(open('$f'));print('8M $f', d['roofline']['k_compact']['ms'], d['verified'])"; done
rm -rf gpurun_out/ab2
BENCH_ARGS="--no-memo-off-run --no-pipelined-run --verify" timeout -k 10 400 bash tools/ab2.sh 4 1 || exit $?
for f in gpurun_out/ab2/c*.json; do python3 -c "import json;d=json.load(open('$f'));print('1M $f', d['roofline']['k_compact']['ms'], d['verified'])"; done
