#!/bin/bash
# Default bench lines after the secondary two-stream region was added: C1 with --verify
# (both batches' results compared, 100k docs vs the oracle), C4 at the 8M-doc shard (no
# room for a second batch: the region is skipped), and the 2-rank shared-GPU test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02bk; mkdir -p $O
timeout -k 10 300 python3 bench.py --verify --steps 20 --warmup 5 --cpu-sample-docs 50000 --cpu-min-seconds 2 > $O/c1.json 2>> $O/err.log || exit $?
python3 -c "import json;d=json.load(open('$O/c1.json'));print('C1', d['value'], d['verified'], d['memo']['memo_off'], d['pipelined'])"
timeout -k 10 600 python3 bench.py --config 4 --docs 8000000 --steps 3 --warmup 1 --no-cpu-baseline --no-memo-off-run > $O/c4_8M.json 2>> $O/err.log || exit $?
python3 -c "import json;d=json.load(open('$O/c4_8M.json'));print('C4 8M', d['value'], d['config']['sub_batches'], d['pipelined'])"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_subbatch.py -x -v --timeout 500 --timeout-method thread -k "two_ranks" > $O/pytest.log 2>&1 || exit $?
tail -1 $O/pytest.log
