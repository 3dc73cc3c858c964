#!/bin/bash
# Times bench.py with each variant library in tokenizer-zig_amd/build/*.so (+ the default).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in tokenizer-zig_amd/tkz/libtkz.so tokenizer-zig_amd/build/*.so; do
  TKZ_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab_$(basename $lib .so).json 2>gpurun_out/ab_$(basename $lib .so).err || exit $?
  echo "$lib $(python3 -c "import json;d=json.load(open('gpurun_out/ab_$(basename $lib .so).json'));print(d['value'], d['roofline']['avg_launch_ms'])")"
done
