# k_encode next-step prefetch: parity tests on the default build, then A/B vs no prefetch (C1, C5, C3)
set -o pipefail
D=gpurun_out/r04o; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_subbatch.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
bash tools/ab.sh 1 5 3
