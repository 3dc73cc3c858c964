#!/bin/bash
# rocprofv3 PMC passes over one command, each counter group in its own run (no tracing
# domains; at most 4 TCC counters per pass: FETCH_SIZE takes 3, WRITE_SIZE 2), plus the
# kernel-source hash of the tree (bench.py takes `traffic` only from a summary whose
# hash matches its own build). Summarise with tools/pmc_summary.py.
#   usage: bash tools/pmc.sh <name> <command with absolute paths...>  -> gpurun_out/pmc_<name>/p<i>/
#   PMC_GROUPS="g1;g2" overrides the default groups (";"-separated).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
NAME=$1
shift
D=$R/gpurun_out/pmc_$NAME
mkdir -p "$D"
python3 -c "import bench; print(bench.kernel_src_hash())" > "$D/src_hash.txt" || exit $?
echo "$*" > "$D/cmd.txt"
DEFAULT="FETCH_SIZE;WRITE_SIZE;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum;\
TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum;TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum TCC_BUBBLE_sum;\
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES;\
GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
IFS=';' read -ra GRP <<< "${PMC_GROUPS:-$DEFAULT}"
cd /tmp && export TMPDIR=/tmp
i=0
for g in "${GRP[@]}"; do
  i=$((i+1))
  echo "$g" > "$D/group$i.txt"
  timeout -s KILL 150 rocprofv3 --pmc $g --kernel-trace --output-format csv -d "$D/p$i" -o run -- "$@" > "$D/p$i.log" 2>&1 || { echo "pass $i ($g) failed: $?"; tail -5 "$D/p$i.log"; exit 1; }
done
echo "pmc $NAME: $i passes"
