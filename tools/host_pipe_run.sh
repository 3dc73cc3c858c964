set -o pipefail
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -k "host_pipeline or golden or edge_cases" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_hp.log 2>&1 || { tail -30 gpurun_out/pytest_hp.log; exit 1; }
tail -1 gpurun_out/pytest_hp.log
for a in "1 1000000 0" "1 1000000 67108864" "1 1000000 33554432" "1 1000000 16777216" "4 1000000 0" "4 1000000 67108864" "4 1000000 33554432"; do
  timeout -k 10 200 python3 tools/bench_host.py $a | tee -a gpurun_out/host_pipe3.jsonl || exit 1
done
