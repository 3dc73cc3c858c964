# very long whole-doc pretokens through the segmented path
set -o pipefail
D=gpurun_out/r04z; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest "tests/test_segments.py::test_gpu_very_long_pretokens" -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
