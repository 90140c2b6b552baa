#!/bin/bash
# Round 4 closing check on the final tree: smoke, the whole GPU suite, the default bench line.
set -e
OUT=gpurun_out/r4_last
mkdir -p $OUT
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
timeout -k 10 400 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
echo done > $OUT/done.txt
