#!/bin/bash
# timing-only prototype: standalone word scan (k_scan) in place of k_encode, grids of 16/32/64 waves per CU
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/aq
for c in 1 2 4; do
  for n in scan32 scan64 scan256; do
    TKZ_LIB=$PWD/tokenizer-zig_amd/build/$n.so timeout -k 10 300 python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-memo-off-run > gpurun_out/aq/c${c}_$n.json 2> gpurun_out/aq/c${c}_$n.err || { tail -20 gpurun_out/aq/c${c}_$n.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/aq/c${c}_$n.json'));r=d['roofline'];print('C$c', '$n', r['avg_launch_ms'], r['other_kernels_ms'])"
  done
done
