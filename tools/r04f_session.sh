set -o pipefail
D=gpurun_out/r04f; mkdir -p $D

timeout -k 10 600 python3 -u -m pytest tests/test_segments.py tests/test_gpu_long.py tests/test_gpu_wide.py tests/test_gpu_host.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
timeout -k 10 300 python3 bench.py --config 6 --steps 3 --warmup 1 --primary-only --no-memo-off-run --no-pipelined-run --no-cpu-baseline > $D/c6.json 2> $D/c6.err || { tail -20 $D/c6.err; exit 1; }
python3 -c "import json;d=json.load(open('$D/c6.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernels']['other_ms'],d['verified']['hash_match'])"
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$D/trace" -o run --output-format csv -- python3 "$R/bench.py" --config 6 --steps 3 --warmup 1 --primary-only --no-memo-off-run --no-pipelined-run --no-cpu-baseline --no-verify > "$R/$D/trace.log" 2>&1 || { tail -20 "$R/$D/trace.log"; exit 1; }
cd "$R"; f=$(find $D/trace -name "*kernel_stats.csv" | head -1); head -20 "$f"
