#!/bin/bash
# k_compact groups of 16 words per lane (1024 words) vs 8 (512)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in wpl16 wpl16m5; do
  TKZ_LIB=$PWD/tokenizer-zig_amd/build/$lib.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_subbatch.py -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_subbatch.py::test_c4_shard_8M > gpurun_out/pytest_r02ag.log 2>&1 || { tail -30 gpurun_out/pytest_r02ag.log; exit 1; }
  tail -1 gpurun_out/pytest_r02ag.log
done
BENCH_ARGS="--no-memo-off-run" timeout -k 10 900 bash tools/ab2.sh 1 3 4 5
for f in gpurun_out/ab2/*_1.json; do python3 -c "import json;d=json.load(open('$f'));print('$f'.split('/')[-1], d['roofline']['k_compact']['ms'])"; done
