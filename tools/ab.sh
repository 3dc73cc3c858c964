#!/bin/bash
# Interleaved A/B timing of variant builds (tools/build_variant.sh -> tokenizer-zig_amd/build/*.so)
# against the default library: every library twice per config, the second time in reverse order.
# Optionally the GPU parity tests on every variant first (TESTS="tests/test_gpu_parity.py ...").
#   usage: [TESTS=...] [BENCH_ARGS=...] bash tools/ab.sh [configs...]    (default 1 2 3 4 5)
# Prints: config, library, GB/s, k_encode ms per launch, deferred / count+scan / compact ms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
[ $# -eq 0 ] && set -- 1 2 3 4 5
libs="tokenizer-zig_amd/tkz/libtkz.so $(ls tokenizer-zig_amd/build/*.so 2>/dev/null)"
if [ -n "$TESTS" ]; then
  for lib in $libs; do
    TKZ_LIB=$PWD/$lib timeout -k 10 900 python3 -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread \
      > gpurun_out/ab/pytest_$(basename $lib .so).log 2>&1 || { tail -30 gpurun_out/ab/pytest_$(basename $lib .so).log; exit 1; }
    echo "$(basename $lib .so): $(tail -1 gpurun_out/ab/pytest_$(basename $lib .so).log)"
  done
fi
rev=$(for l in $libs; do echo $l; done | tac | tr '\n' ' ')
for c in "$@"; do
  for rep in 1 2; do
    # ABBA: the second repetition runs the libraries in reverse order (a process's position
    # in the sequence moved k_compact by up to 7 % on C4 in r03m / r03p)
    order=$libs; [ $rep = 2 ] && order=$rev
    for lib in $order; do
      n=$(basename $lib .so)
      o=gpurun_out/ab/c${c}_${n}_${rep}
      TKZ_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline \
        --primary-only --no-memo-off-run --no-pipelined-run ${BENCH_ARGS} > $o.json 2> $o.err || { tail -20 $o.err; exit 1; }
      python3 -c "import json;d=json.load(open('$o.json'));k=d['roofline']['kernels'];print('C$c', '$n', round(d['value']/1e3,1), k['k_encode']['avg_launch_ms'], k['other_ms'], k['k_compact']['ms'])"
    done
  done
done
