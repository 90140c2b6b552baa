#!/bin/bash
# One GPU-box session: the GPU test suite, smoke(), then the default bench line.
# usage: tools/gpu_round.sh <tag> [pytest -k expr]
set -e
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
K=${2:-}
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KARG[@]}" \
  > $OUT/gputest.log 2>&1
tail -3 $OUT/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
