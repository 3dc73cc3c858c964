# k_encode SALU attribution: SQ instruction counts of the default build and the ablation
# builds (scan only, memo with misses dropped, no rounds, no doc walk, scalar doc walk) on
# C1, and the default on C5
set -o pipefail
LIBS="tokenizer-zig_amd/tkz/libtkz.so tokenizer-zig_amd/build/scalardocs.so tokenizer-zig_amd/build/abl6.so tokenizer-zig_amd/build/abl4.so tokenizer-zig_amd/build/abl2.so tokenizer-zig_amd/build/nodocwalk.so" CONFIG=1 bash tools/bisect_pmc.sh && \
LIBS="tokenizer-zig_amd/tkz/libtkz.so" CONFIG=5 bash tools/bisect_pmc.sh
