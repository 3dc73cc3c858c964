# k_seg_first ablations on C6 (timing only): kernel traces of the default build, no
# boundary checks (segf1), no memo lookups (segf2)
set -o pipefail
R=$(pwd); D=$R/gpurun_out/r04k; mkdir -p $D; cd /tmp && export TMPDIR=/tmp
for v in tkz/libtkz build/segf1 build/segf2; do
  n=$(basename $v)
  TKZ_LIB=$R/tokenizer-zig_amd/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/$n -o run --output-format csv -- python3 $R/bench.py --config 6 --steps 2 --warmup 1 --primary-only --no-memo-off-run --no-pipelined-run --no-cpu-baseline --no-verify > $D/$n.log 2>&1 || { tail -5 $D/$n.log; exit 1; }
  f=$(find $D/$n -name "*kernel_stats.csv" | head -1); grep -E "k_seg_first|k_seg_out|k_seg_init" "$f" | cut -d, -f1-4
done
