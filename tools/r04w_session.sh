# segmented-path variants on C6: the seg tests on the check-preload build, then kernel traces
# of the default build, check preload, replay width 6 and 8
set -o pipefail
R=$(pwd); D=$R/gpurun_out/r04w; mkdir -p $D
TKZ_LIB=$R/tokenizer-zig_amd/build/preload.so timeout -k 10 600 python3 -u -m pytest tests/test_segments.py tests/test_gpu_long.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest_preload.log 2>&1 || { tail -30 $D/pytest_preload.log; exit 1; }
tail -1 $D/pytest_preload.log
cd /tmp && export TMPDIR=/tmp
for v in tkz/libtkz build/preload build/kp6 build/kp8; do
  n=$(basename $v)
  TKZ_LIB=$R/tokenizer-zig_amd/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/$n -o run --output-format csv -- python3 $R/bench.py --config 6 --steps 3 --warmup 1 --primary-only --no-memo-off-run --no-pipelined-run --no-cpu-baseline --no-verify > $D/$n.log 2>&1 || { tail -5 $D/$n.log; exit 1; }
  python3 - $D/$n <<'PY'
import csv,sys,glob
f=glob.glob(sys.argv[1]+'/**/*kernel_stats.csv',recursive=True)[0]
tot=0
for r in csv.DictReader(open(f)):
    if 'k_seg' in r['Name']:
        print(sys.argv[1].split('/')[-1], r['Name'].split('(')[0], r['Calls'], round(float(r['AverageNs'])/1e6,3))
PY
done
