# sub-batch tests including the segmented path (C6) and wide tables (C7)
set -o pipefail
D=gpurun_out/r04z; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest "tests/test_gpu_subbatch.py::test_sub_batches_exact" -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
