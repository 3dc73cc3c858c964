#!/bin/bash
# PMC traffic passes (request-size read counters, WRITE_SIZE) of the default library and the
# variant builds named in $VARIANTS (tokenizer-zig_amd/build/<name>.so), C1 primary region.
#   usage: VARIANTS="cabl1 cabl2" bash tools/pmc_variants.sh
set -o pipefail
R=$(pwd)
for v in libtkz ${VARIANTS}; do
  if [ $v = libtkz ]; then L=$R/tokenizer-zig_amd/tkz/libtkz.so; else L=$R/tokenizer-zig_amd/build/$v.so; fi
  TKZ_LIB=$L PMC_GROUPS="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum;WRITE_SIZE" \
    bash tools/pmc.sh ${TAG:-var}_$v python3 $R/bench.py --steps 2 --warmup 0 --primary-only --no-memo-off-run --no-pipelined-run --no-cpu-baseline --no-verify --no-host-e2e || exit 1
done
