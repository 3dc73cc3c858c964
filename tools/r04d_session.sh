set -o pipefail
D=gpurun_out/r04d; mkdir -p $D
for lib in tokenizer-zig_amd/tkz/libtkz.so tokenizer-zig_amd/build/seg_minb4.so tokenizer-zig_amd/tkz/libtkz.so tokenizer-zig_amd/build/seg_minb4.so; do
  TKZ_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --config 6 --steps 3 --warmup 1 --primary-only --no-memo-off-run --no-pipelined-run --no-cpu-baseline --no-verify > $D/c6.json 2> $D/c6.err || { tail -20 $D/c6.err; exit 1; }
  python3 -c "import json;d=json.load(open('$D/c6.json'));print('$lib',d['value'],d['ms_per_step'],d['roofline']['kernels']['other_ms'])"
done
TKZ_LIB=$PWD/tokenizer-zig_amd/build/segstats_minb4.so timeout -k 10 300 python3 tools/seg_phases.py 200000 > $D/phases4.txt 2>&1 || { tail -20 $D/phases4.txt; exit 1; }
cat $D/phases4.txt
