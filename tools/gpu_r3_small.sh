#!/bin/bash
# Small-batch study: GPU suite subset for the one-launch path, the callers
# study, and a kernel trace of 4k-topic host batches.
# usage: tools/gpu_r3_small.sh <tag>
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
tail -2 $OUT/gputest.log
timeout -k 10 300 python3 -u tools/callers_study.py > $OUT/callers.jsonl 2> $OUT/callers.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/lat -o run --output-format csv -- \
  python3 -u tools/latency_trace.py --batch 4096 --reps 60 > $OUT/lat.log 2>&1
