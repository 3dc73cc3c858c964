#!/bin/bash
# deferred BPE split by length (12-symbol short class) vs one launch
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in tokenizer-zig_amd/tkz/libtkz.so tokenizer-zig_amd/build/s4.so; do
  TKZ_LIB=$PWD/$lib timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_subbatch.py -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_subbatch.py::test_c4_shard_8M > gpurun_out/pytest_r02af.log 2>&1 || { tail -30 gpurun_out/pytest_r02af.log; exit 1; }
  tail -1 gpurun_out/pytest_r02af.log
done
BENCH_ARGS="--no-memo-off-run" timeout -k 10 900 bash tools/ab2.sh 1 2 5
