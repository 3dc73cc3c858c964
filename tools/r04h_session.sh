# full GPU suite, then the C6 segmented-path session and the k_encode PMC attribution
set -o pipefail
mkdir -p gpurun_out/r04h
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04h/pytest.log 2>&1 || { tail -30 gpurun_out/r04h/pytest.log; exit 1; }
tail -1 gpurun_out/r04h/pytest.log
bash tools/r04f_session.sh > gpurun_out/r04f_out.txt 2>&1 || { tail -20 gpurun_out/r04f_out.txt; exit 1; }
tail -3 gpurun_out/r04f_out.txt
bash tools/r04g_session.sh
