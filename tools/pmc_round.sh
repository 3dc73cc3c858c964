#!/bin/bash
# PMC passes on k_encode (each counter group in its own rocprofv3 run; no tracing domains).
# usage: TAG=r01x bash tools/pmc_round.sh ["GROUP1" "GROUP2" ...]   (TKZ_LIB selects a variant)
# FETCH_SIZE and WRITE_SIZE must be in separate passes (together they exceed the hardware's
# counter budget and rocprofv3 aborts).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); TAG=${TAG:-r01}
mkdir -p gpurun_out/pmc_${TAG}
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 2 --warmup 0 --no-cpu-baseline ${BENCH_ARGS}"
if [ $# -eq 0 ]; then
  set -- "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
         "FETCH_SIZE" "WRITE_SIZE" \
         "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
fi
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_${TAG}/p$i" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_${TAG}/p$i.log" 2>&1 || exit $?
done
