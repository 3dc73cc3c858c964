# diagnosis of the segmented path's C1-under-ByteLevel mismatch: default library and
# variants (no k_seg_first, no W = 32 lane encode)
set -o pipefail
D=gpurun_out/r04i; mkdir -p $D
timeout -k 10 300 python3 -u tools/long_diag.py > $D/default.txt 2>&1 || { tail -20 $D/default.txt; exit 1; }
for v in noseg1st now32; do
  TKZ_LIB=$(pwd)/tokenizer-zig_amd/build/$v.so timeout -k 10 300 python3 -u tools/long_diag.py > $D/$v.txt 2>&1 || { tail -20 $D/$v.txt; exit 1; }
done
head -50 $D/*.txt
