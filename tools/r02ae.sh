#!/bin/bash
# timing-only: k_encode without the scan past each chunk's end (abl8) vs the default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abl8
for rep in 1 2; do for lib in libtkz abl8; do
  f=tokenizer-zig_amd/tkz/libtkz.so; [ $lib = abl8 ] && f=tokenizer-zig_amd/build/abl8.so
  for c in 1 4 5; do
    TKZ_LIB=$PWD/$f timeout -k 10 300 python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-memo-off-run > gpurun_out/abl8/${lib}_c$c.json 2> gpurun_out/abl8/${lib}_c$c.err || { tail -5 gpurun_out/abl8/${lib}_c$c.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/abl8/${lib}_c$c.json'));r=d['roofline'];print('C$c $lib', r['avg_launch_ms'], d['ms_per_step'])"
  done
done; done
