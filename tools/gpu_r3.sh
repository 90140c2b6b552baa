#!/bin/bash
# Round-3 GPU session: the GPU suite, smoke(), the default bench line, then a
# kernel trace of 4k-topic host batches (tools/latency_trace.py) -- where a
# small batch's time goes.  Any failing / timed-out step ends the script.
# usage: tools/gpu_r3.sh <tag> [--no-tests]
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "--no-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
  tail -2 $OUT/gputest.log
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
fi
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/lat -o run --output-format csv -- \
  python3 -u tools/latency_trace.py --batch 4096 --reps 60 > $OUT/lat.log 2>&1
