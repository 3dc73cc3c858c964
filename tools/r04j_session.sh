# PMC of the segmented path's kernels on C6: SQ instruction / wait counters, then L2
set -o pipefail
rm -rf gpurun_out/bisect
LIBS="tokenizer-zig_amd/tkz/libtkz.so" CONFIG=6 bash tools/bisect_pmc.sh && \
LIBS="tokenizer-zig_amd/tkz/libtkz.so" CONFIG=6 SUFFIX=_tcc COUNTERS="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" bash tools/bisect_pmc.sh && \
python3 tools/bisect_summary.py gpurun_out/bisect k_seg > gpurun_out/bisect/seg_summary.txt
