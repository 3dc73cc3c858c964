#!/bin/bash
# Alternating A/B timing: every library in tokenizer-zig_amd/build/*.so plus the default, run twice
# each in interleaved order, for the configs given (default 1 2 3 4). Prints config, lib, GB/s, k_encode ms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab2
[ $# -eq 0 ] && set -- 1 2 3 4
libs="tokenizer-zig_amd/tkz/libtkz.so $(ls tokenizer-zig_amd/build/*.so 2>/dev/null)"
for c in "$@"; do
  for rep in 1 2; do
    for lib in $libs; do
      n=$(basename $lib .so)
      o=gpurun_out/ab2/c${c}_${n}_${rep}
      TKZ_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $o.json 2> $o.err || { tail -20 $o.err; exit 1; }
      python3 -c "import json;d=json.load(open('$o.json'));r=d['roofline'];print('C$c', '$n', round(d['value']/1e3,1), r['avg_launch_ms'], r['other_kernels_ms'])"
    done
  done
done
