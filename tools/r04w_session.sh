# k_seg_first: replay pairs probed 4 / 6 / 8 at a time (C6 kernel traces)
set -o pipefail
R=$(pwd); D=$R/gpurun_out/r04w; mkdir -p $D; cd /tmp && export TMPDIR=/tmp
for v in tkz/libtkz build/kp6 build/kp8; do
  n=$(basename $v)
  TKZ_LIB=$R/tokenizer-zig_amd/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/$n -o run --output-format csv -- python3 $R/bench.py --config 6 --steps 3 --warmup 1 --primary-only --no-memo-off-run --no-pipelined-run --no-cpu-baseline --no-verify > $D/$n.log 2>&1 || { tail -5 $D/$n.log; exit 1; }
  python3 - $D/$n <<'PY'
import csv,sys,glob
f=glob.glob(sys.argv[1]+'/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'k_seg' in r['Name']: print(sys.argv[1].split('/')[-1], r['Name'].split('(')[0], r['Calls'], round(float(r['AverageNs'])/1e6,3))
PY
done
