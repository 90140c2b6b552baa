#!/bin/bash
# The GPU test suite only (optionally a -k selection), verbose, per-test timeouts.
# usage: tools/gpu_tests.sh <tag> [pytest -k expr]
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
if [ -n "$2" ]; then KARG=(-k "$2"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread "${KARG[@]}" \
  > $OUT/gputest.log 2>&1
tail -3 $OUT/gputest.log
