#!/bin/bash
# Builds tokenizer-zig_amd/build/<name>.so from the working tree (or from a git revision
# with REV=<rev>) with extra -D flags, for A/B timing with tools/ablate.sh.
# usage: [REV=HEAD] bash tools/build_variant.sh <name> [-DFLAG ...]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
src=tokenizer-zig_amd/csrc
if [ -n "$REV" ]; then
  tmp=$(mktemp -d)
  mkdir -p "$tmp/include" "$tmp/x/csrc"   # csrc/../../include as in the tree
  for f in $(git ls-tree --name-only "$REV" tokenizer-zig_amd/csrc/); do git show "$REV:$f" > "$tmp/x/csrc/$(basename $f)"; done
  git show "$REV:include/tkz.h" > "$tmp/include/tkz.h"
  src="$tmp/x/csrc"
fi
mkdir -p tokenizer-zig_amd/build
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DTKZ_MAXB=24 -Wno-unused-result -Wno-unused-value \
  -I include "$@" -shared -o tokenizer-zig_amd/build/$name.so \
  $src/encode.hip $src/decode.hip $src/pad.hip $src/span.hip $src/tokenizer.cpp
