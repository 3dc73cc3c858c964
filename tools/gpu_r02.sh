#!/bin/bash
# Round-2 GPU session: smoke -> GPU tests -> bench lines (C1 default, C5, other configs,
# C4 at 8M docs per GPU) -> rocprofv3 kernel trace of the default bench command.
# Every GPU step has its own time limit; steps are chained with && (stop at the first failure).
# usage: TAG=r02a [PYTEST_ARGS=...] [SKIP_TESTS=1] [SKIP_BENCH=1] [SKIP_PROF=1] bash tools/gpu_r02.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
TAG=${TAG:-r02}
O=gpurun_out/$TAG
mkdir -p $O
echo "host: $(nproc) cpus; $(python3 -c 'import os;print(len(os.sched_getaffinity(0)))') in affinity; cgroup $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)" > $O/host.txt
step() { echo "[$(date +%T)] $*" >> $O/steps.log; }
run_tests() {
  [ -n "$SKIP_TESTS" ] && return 0
  step smoke
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || return $?
  step pytest
  timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1 || return $?
}
run_bench() {
  [ -n "$SKIP_BENCH" ] && return 0
  step bench c1
  timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $O/bench_c1.json 2> $O/bench.err || return $?
  step bench c5
  timeout -k 10 300 python3 bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5.json 2>> $O/bench.err || return $?
  for c in 2 3 4; do
    step bench c$c
    timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 2 --cpu-sample-docs 100000 --cpu-min-seconds 4 > $O/bench_c$c.json 2>> $O/bench.err || return $?
  done
  step bench c4 8M
  timeout -k 10 900 python3 bench.py --config 4 --docs 8000000 --steps 3 --warmup 1 --no-cpu-baseline --no-memo-off-run > $O/bench_c4_8M.json 2>> $O/bench.err || return $?
}
run_prof() {
  [ -n "$SKIP_PROF" ] && return 0
  step rocprof
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-memo-off-run --no-pipelined-run > "$R/$O/prof.log" 2>&1)
}
run_tests && run_bench && run_prof
rc=$?
step "done rc=$rc"
exit $rc
