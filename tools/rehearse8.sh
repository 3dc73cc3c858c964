#!/bin/bash
# The 8-rank bench command on ONE GPU (bench.py --gpus 8 --share-gpu): every rank's default
# regions except that the 8M-doc C4 shard is replaced by 1M docs and every workspace capped
# at 3 GiB (eight ranks of the real 8-GPU run's C4 shard need ~8 x 100 GB of HBM), oracle
# threads split across the ranks. Output: gpurun_out/<tag>/bench8.json + wall time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04r}; D=gpurun_out/$TAG; mkdir -p $D
t0=$(date +%s)
timeout -k 10 1100 python3 bench.py --gpus 8 --share-gpu --max-workspace-gb 3 \
  --secondary 2:1000000,3:1000000,5:1000000,4:1000000,6:1000000,7:1000000 \
  > $D/bench8.json 2> $D/bench8.err || { tail -30 $D/bench8.err; exit 1; }
echo "wall_s $(( $(date +%s) - t0 ))" | tee $D/bench8_wall.txt
python3 -c "
import json;d=json.load(open('$D/bench8.json'))
print('value', d['value'], 'ranks_failed', d['verified']['ranks_failed'], 'n_gpus', d['n_gpus'])
for k,v in (d.get('secondary') or {}).items(): print(k, v['value'], v['ranks_failed'], v['verified'])
print('host_e2e', (d.get('host_e2e') or {}).get('value'), (d.get('host_e2e') or {}).get('ranks_failed'))"
