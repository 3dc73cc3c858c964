#!/bin/bash
# PMC passes on bench.py for the default library and each variant in tokenizer-zig_amd/build/*.so
# usage: TAG=x bash tools/pmc_ab.sh "GROUP1" "GROUP2" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); TAG=${TAG:-ab}
mkdir -p gpurun_out/pmc_${TAG}
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 2 --warmup 0 --no-cpu-baseline ${BENCH_ARGS}"
for lib in "$R"/tokenizer-zig_amd/tkz/libtkz.so "$R"/tokenizer-zig_amd/build/*.so; do
  n=$(basename $lib .so); i=0
  for grp in "$@"; do
    i=$((i+1))
    TKZ_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_${TAG}/${n}/p$i" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_${TAG}/${n}_p$i.log" 2>&1 || exit $?
  done
done
