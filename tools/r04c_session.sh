set -o pipefail
D=gpurun_out/r04c; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest tests/test_segments.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
TKZ_LIB=$PWD/tokenizer-zig_amd/build/segstats.so timeout -k 10 300 python3 tools/seg_phases.py 200000 > $D/phases.txt 2>&1 || { tail -20 $D/phases.txt; exit 1; }
cat $D/phases.txt
timeout -k 10 300 python3 bench.py --config 6 --steps 3 --warmup 1 --primary-only --no-memo-off-run --no-pipelined-run --no-cpu-baseline --no-verify > $D/c6.json 2> $D/c6.err || { tail -20 $D/c6.err; exit 1; }
python3 -c "import json;d=json.load(open('$D/c6.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernels']['other_ms'])"
