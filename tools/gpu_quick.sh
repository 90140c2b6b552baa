#!/bin/bash
# GPU parity tests + walk timing on the main configs (no profiler).
# usage: tools/gpu_quick.sh <tag> [--no-tests]
set -e
TAG=$1; shift
OUT=gpurun_out/quick_$TAG
mkdir -p $OUT
if [ "$1" != "--no-tests" ]; then
  timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
fi
for c in c3 c2nm c1; do
  timeout -k 10 180 python3 -u tools/profile_walk.py --config $c --batches 10 >> $OUT/timing.txt 2>&1
done
