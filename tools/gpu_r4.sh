#!/bin/bash
# Round 4: the default bench line, a driver-shaped short line, then the whole GPU suite.
# usage: tools/gpu_r4.sh <tag> [--no-tests]
set -e
OUT=gpurun_out/r4_$1
mkdir -p $OUT
timeout -k 10 400 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --latency-batches 0 --concurrency 0 --no-cpu \
  > $OUT/bench_20.json 2> $OUT/bench_20.err
if [ "$2" != "--no-tests" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
fi
echo done > $OUT/done.txt
