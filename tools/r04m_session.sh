# wide-id path: tests, then C7 as the primary region with a kernel trace
set -o pipefail
D=gpurun_out/r04m; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_wide.py tests/test_gpu_parity.py tests/test_gpu_long.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
timeout -k 10 300 python3 bench.py --config 7 --steps 5 --warmup 1 --primary-only --no-memo-off-run --no-pipelined-run --no-cpu-baseline > $D/c7.json 2> $D/c7.err || { tail -20 $D/c7.err; exit 1; }
python3 -c "import json;d=json.load(open('$D/c7.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernels'].get('k_encode',{}).get('ms'),d['verified'])"
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$D/trace" -o run --output-format csv -- python3 "$R/bench.py" --config 7 --steps 3 --warmup 1 --primary-only --no-memo-off-run --no-pipelined-run --no-cpu-baseline --no-verify > "$R/$D/trace.log" 2>&1 || { tail -20 "$R/$D/trace.log"; exit 1; }
cd "$R"; f=$(find $D/trace -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -12
