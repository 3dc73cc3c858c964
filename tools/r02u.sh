#!/bin/bash
# k_compact group size / occupancy variants (build/*.so) vs the default: parity of the
# variants on the bench configs, then interleaved A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in tokenizer-zig_amd/build/wpl4.so tokenizer-zig_amd/build/wpl4m8.so; do
  TKZ_LIB=$PWD/$lib timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bench or golden or edge" > gpurun_out/pytest_r02u.log 2>&1 || { tail -30 gpurun_out/pytest_r02u.log; exit 1; }
  tail -1 gpurun_out/pytest_r02u.log
done
BENCH_ARGS="--no-memo-off-run" timeout -k 10 900 bash tools/ab2.sh 1 3 4 5
