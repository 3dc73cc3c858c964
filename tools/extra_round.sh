#!/bin/bash
# Larger-shard C4 bench and host-buffer (PCIe-inclusive) rates of every config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --config 4 --docs 4000000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4_4M.json 2> gpurun_out/bench_c4_4M.err || { tail -20 gpurun_out/bench_c4_4M.err; exit 1; }
cat gpurun_out/bench_c4_4M.json
for c in 1 2 3 4; do
  timeout -k 10 300 python3 tools/bench_host.py $c 1000000 | tee -a gpurun_out/host_all.jsonl || exit 1
done
