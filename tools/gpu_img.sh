#!/bin/bash
# Image lock split: GPU suite, then 4k callers with and without churn.
# usage: tools/gpu_img.sh <tag>
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
tail -1 $OUT/gputest.log
timeout -k 10 200 python3 -u tools/conc_sweep.py --churn 0,256 --threads 8,16 > $OUT/sweep.jsonl 2>> $OUT/sweep.err
