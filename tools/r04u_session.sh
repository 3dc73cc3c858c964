# the default bench line alone (host region after the primary)
set -o pipefail
D=gpurun_out/r04u; mkdir -p $D
timeout -k 10 900 python3 bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$D/bench.json'));print(d['value'],d['roofline']['traffic_ratio'],d['host_e2e']['value'],d['host_e2e']['ms_per_call'],d['host_e2e']['frac_of_d2h_floor'])"
