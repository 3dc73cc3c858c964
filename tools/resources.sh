#!/bin/bash
# Per-kernel register / LDS / occupancy summary of encode.hip (extra -D flags pass through).
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DTKZ_MAXB=24 -I include "$@" \
  -Rpass-analysis=kernel-resource-usage -c tokenizer-zig_amd/csrc/encode.hip -o /tmp/tkz_res.o 2>&1 |
  sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass.*//' | awk -F': ' '
    $1=="Function Name" {n=substr($2,1,58)}
    $1=="VGPRs" {v=$2} $1=="TotalSGPRs" {s=$2} $1=="ScratchSize [bytes/lane]" {sc=$2}
    $1=="Occupancy [waves/SIMD]" {o=$2}
    $1=="LDS Size [bytes/block]" {printf "%-58s VGPR %3s SGPR %3s scratch %3s occ %s LDS %s\n", n, v, s, sc, o, $2}'
