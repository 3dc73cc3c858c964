#!/bin/bash
# timing-only ablations of k_encode (C1): abl5 = memo probes without memory access,
# abl6 = scan + word ring only (no dispatch), abl7 = scan without ring writes. Outputs are
# not valid (no verification); k_encode time is what is read.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abl
for rep in 1 2; do
for lib in head abl5 abl6 abl7; do
  f=tokenizer-zig_amd/build/$lib.so
  TKZ_LIB=$PWD/$f timeout -k 10 300 python3 bench.py --config 1 --steps 5 --warmup 1 --no-cpu-baseline --no-memo-off-run > gpurun_out/abl/$lib.json 2> gpurun_out/abl/$lib.err || { tail -5 gpurun_out/abl/$lib.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/abl/$lib.json'));r=d['roofline'];print('$lib', r['avg_launch_ms'], r['k_compact']['ms'], d['ms_per_step'])"
done
done
