#!/bin/bash
# bench.py with two batches in flight on two streams (default when they fit) vs one stream,
# interleaved, C1 / C5 / C4; then the default C1 command with --verify (both streams'
# results compared and the first 100k docs vs the oracle) and the 2-rank shared-GPU test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02bj; mkdir -p $O
for c in 1 5 4; do
  for rep in 1 2; do
    for s in 1 2; do
      timeout -k 10 300 python3 bench.py --config $c --streams $s --steps 20 --warmup 3 --no-cpu-baseline --no-memo-off-run --no-pipelined-run > $O/c${c}_s${s}_${rep}.json 2>> $O/err.log || exit $?
      python3 -c "import json;d=json.load(open('$O/c${c}_s${s}_${rep}.json'));r=d['roofline'];print('C$c streams=$s', round(d['value']/1e3,1), d['ms_per_step'], r['avg_launch_ms'], r['k_compact']['ms'])"
    done
  done
done
timeout -k 10 300 python3 bench.py --verify --steps 20 --warmup 5 --cpu-sample-docs 50000 --cpu-min-seconds 2 > $O/c1_default_verify.json 2>> $O/err.log || exit $?
python3 -c "import json;d=json.load(open('$O/c1_default_verify.json'));print('default C1', d['value'], d['config']['streams'], d['verified'], d['memo']['memo_off'], d['pipelined'])"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_subbatch.py -x -v --timeout 500 --timeout-method thread -k "two_ranks" > $O/pytest.log 2>&1 || exit $?
tail -1 $O/pytest.log
