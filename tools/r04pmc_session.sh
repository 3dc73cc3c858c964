# C1 PMC passes at the current source (bench.py's traffic field reads the committed summary)
set -o pipefail
R=$(pwd)
bash tools/pmc.sh ${TAG:-r04final} python3 "$R/bench.py" --steps 2 --warmup 0 --primary-only --no-memo-off-run \
  --no-pipelined-run --no-cpu-baseline --no-verify
