#!/bin/bash
# PMC passes over the default bench command (C1), each counter group in its own rocprofv3
# run (no tracing domains), plus the kernel-source hash of the tree that ran them
# (bench.py reports `traffic` only from a summary whose hash matches its own build).
# usage: TAG=r02x bash tools/pmc_r02.sh ["GROUP1" "GROUP2" ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); TAG=${TAG:-r02}
D=gpurun_out/pmc_${TAG}
mkdir -p $D
python3 -c "import bench; print(bench.kernel_src_hash())" > $D/src_hash.txt || exit $?
ARGS="--steps 2 --warmup 0 --no-cpu-baseline --no-memo-off-run --no-pipelined-run ${BENCH_ARGS}"
echo "bench.py $ARGS" > $D/cmd.txt
if [ $# -eq 0 ]; then
  set -- "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
         "FETCH_SIZE" "WRITE_SIZE" \
         "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum"
fi
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  echo "$grp" > "$R/$D/group$i.txt"
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$R/$D/p$i" -o run -- python3 "$R/bench.py" $ARGS > "$R/$D/p$i.log" 2>&1 || exit $?
done
