# new parity tests: dense doc boundaries, C2 docs under ByteLevel + Lowercase (segmented on/off)
set -o pipefail
D=gpurun_out/r04v; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py::test_dense_doc_boundaries tests/test_segments.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
