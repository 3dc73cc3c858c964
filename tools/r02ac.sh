#!/bin/bash
# multi-GPU host batch (virtual devices on one GPU), tkz_opts, then the full GPU suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_multi.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r02ac_multi.log 2>&1 || { tail -40 gpurun_out/pytest_r02ac_multi.log; exit 1; }
tail -3 gpurun_out/pytest_r02ac_multi.log
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_subbatch.py::test_c4_shard_8M > gpurun_out/pytest_r02ac.log 2>&1 || { tail -40 gpurun_out/pytest_r02ac.log; exit 1; }
tail -1 gpurun_out/pytest_r02ac.log
