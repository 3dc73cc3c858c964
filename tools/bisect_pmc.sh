#!/bin/bash
# Instruction counts per kernel launch (SQ_INSTS_VALU / SALU / LDS, wave cycles) of the
# default library and of every tools/build_variant.sh build, one rocprofv3 --pmc pass each
# over a short primary-region bench; summarised by tools/bisect_summary.py.
#   usage: [CONFIG=1] [COUNTERS=...] [SUFFIX=_tcc] [LIBS="a.so b.so"] bash tools/bisect_pmc.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); C=${CONFIG:-1}
# one pass; SQ counters by default, e.g. COUNTERS="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_HIT_sum TCC_MISS_sum"
COUNTERS=${COUNTERS:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAVES"}
SUFFIX=${SUFFIX:-}
mkdir -p gpurun_out/bisect
for lib in ${LIBS:-tokenizer-zig_amd/tkz/libtkz.so $(ls tokenizer-zig_amd/build/*.so 2>/dev/null)}; do
  n=$(basename $lib .so)
  (cd /tmp && export TMPDIR=/tmp TKZ_LIB=$R/$lib && timeout -s KILL 150 rocprofv3 --pmc $COUNTERS \
    -d $R/gpurun_out/bisect/c${C}_$n$SUFFIX -o run --output-format csv -- \
    python3 $R/bench.py --config $C --steps 2 --warmup 0 --primary-only --no-memo-off-run --no-pipelined-run \
    --no-cpu-baseline --no-verify > $R/gpurun_out/bisect/c${C}_$n$SUFFIX.log 2>&1) || { tail -5 gpurun_out/bisect/c${C}_$n$SUFFIX.log; exit 1; }
  echo "pmc c$C $n done"
done
