# host path: the replica's tokenizer sequence with a settle pause, and the bench host region
set -o pipefail
D=gpurun_out/r04n; mkdir -p $D
timeout -k 10 400 python3 tools/host_replica.py > $D/replica.txt 2>&1 || { tail -5 $D/replica.txt; exit 1; }
cat $D/replica.txt
A="--no-memo-off-run --no-pipelined-run --no-cpu-baseline --steps 2 --warmup 1 --secondary none"
timeout -k 10 300 python3 bench.py $A > $D/host_settled.json 2> $D/host_settled.err || { tail -5 $D/host_settled.err; exit 1; }
python3 -c "import json;d=json.load(open('$D/host_settled.json'))['host_e2e'];print('bench settled',d['value'],d['ms_per_call'],d['ms_per_call_pinned_input'],d['timeline_pageable_ms']['d2h_span_ms'],d['frac_of_d2h_floor'])"
