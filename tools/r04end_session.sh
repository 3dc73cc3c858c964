# end-of-round check at the final tree: smoke, every GPU test, the default bench line
set -o pipefail
D=gpurun_out/${TAG:-r04end}; mkdir -p $D
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
timeout -k 10 900 python3 bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$D/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['traffic_ratio'],{k:v['value'] for k,v in d['secondary'].items()},d['host_e2e']['value'])"
