#!/bin/bash
# two batches in flight on two streams with k_encode leaving room (20 = full 5 waves/SIMD, 16, 12 blocks per CU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for lib in tkz/libtkz build/per16 build/per12; do
  f=$PWD/tokenizer-zig_amd/$lib.so; [ "$lib" = tkz/libtkz ] || f=$PWD/tokenizer-zig_amd/$lib.so
  echo "== $lib"
  for c in 1 5; do TKZ_LIB=$f timeout -k 10 300 python3 tools/bench_streams.py $c 2 20 || exit $?; done
done
