#!/bin/bash
# the whole 64M-doc C4 stream on one GPU, shard by shard, against the oracle's hashes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1100 python3 -u -m pytest tests/test_gpu_subbatch.py -m gpu -v -s --timeout 900 --timeout-method thread -k "c4_stream or c4_shard" 2>&1 | tee gpurun_out/pytest_r02aj.log | grep -E "PASSED|FAILED|hashes match|Error|error" 
