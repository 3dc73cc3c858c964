#!/bin/bash
# VALU/SALU/LDS instruction counts per k_encode launch for the timing-only ablations
# (head = full kernel, abl5 = memo probes without memory, abl6 = scan + ring only, abl7 =
# scan without ring), one PMC pass each (C1 bench command).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); D=gpurun_out/pmc_abl; mkdir -p $D
cd /tmp && export TMPDIR=/tmp
for lib in head abl5 abl6 abl7; do
  TKZ_LIB=$R/tokenizer-zig_amd/build/$lib.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_ANY --kernel-trace --output-format csv -d "$R/$D/$lib" -o run -- python3 "$R/bench.py" --steps 2 --warmup 0 --no-cpu-baseline --no-memo-off-run > "$R/$D/$lib.log" 2>&1 || exit $?
done
