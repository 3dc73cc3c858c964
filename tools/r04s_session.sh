# round-4 measurement session: smoke, every GPU test, the default bench line, its kernel
# trace, C1 PMC passes (tools/pmc.sh), then C6 and C7 SQ counters (tools/bisect_pmc.sh)
set -o pipefail
TAG=${TAG:-r04s} bash tools/gpu_session.sh || exit 1
rm -rf gpurun_out/bisect
LIBS="tokenizer-zig_amd/tkz/libtkz.so" CONFIG=6 bash tools/bisect_pmc.sh && \
LIBS="tokenizer-zig_amd/tkz/libtkz.so" CONFIG=7 bash tools/bisect_pmc.sh && \
python3 tools/bisect_summary.py gpurun_out/bisect k_seg k_encode k_compact k_bpe > gpurun_out/bisect/summary.txt
