#!/bin/bash
# timing-only: in-lane prototype (proto) vs misses-dropped ablation (abl4), BPE configs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/proto
for rep in 1 2; do for lib in abl4 proto; do for c in 1 4 5; do
  TKZ_LIB=$PWD/tokenizer-zig_amd/build/$lib.so timeout -k 10 300 python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-memo-off-run > gpurun_out/proto/${lib}_c$c.json 2> gpurun_out/proto/${lib}_c$c.err || { tail -5 gpurun_out/proto/${lib}_c$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/proto/${lib}_c$c.json'));r=d['roofline'];print('C$c $lib', r['avg_launch_ms'], d['ms_per_step'], d['config']['tokens_per_gpu'])"
done; done; done
