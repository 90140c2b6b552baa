#!/bin/bash
# Round-end check: GPU suite, smoke(), the default bench line.  usage: tools/gpu_final_check.sh <tag>
set -e
OUT=gpurun_out/check_$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
tail -1 $OUT/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
