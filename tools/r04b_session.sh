set -o pipefail
D=gpurun_out/r04b; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests/test_segments.py tests/test_gpu_long.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 300 python3 bench.py --config 6 --steps 3 --warmup 1 --primary-only --no-memo-off-run --no-pipelined-run --no-cpu-baseline > $D/c6.json 2> $D/c6.err || { tail -20 $D/c6.err; exit 1; }
timeout -k 10 300 python3 bench.py --config 6 --steps 3 --warmup 1 --primary-only --no-memo-off-run --no-pipelined-run --no-cpu-baseline --no-long-segments > $D/c6_noseg.json 2> $D/c6_noseg.err || { tail -20 $D/c6_noseg.err; exit 1; }
timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --no-memo-off-run --no-pipelined-run --no-cpu-baseline --secondary 6:1000000 > $D/c1_host.json 2> $D/c1_host.err || { tail -20 $D/c1_host.err; exit 1; }
echo done
