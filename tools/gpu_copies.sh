#!/bin/bash
# Table copies (tm_options.copies): GPU suite, C5 bench lines with 1 / 2 / 3
# copies, and 4k callers with churn on a 2-copy index.  usage: tools/gpu_copies.sh <tag>
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
tail -1 $OUT/gputest.log
for c in 1 2 3; do
  timeout -k 10 400 python -u bench.py --config c5 --copies $c --no-cpu --latency-batches 0 --concurrency 0 > $OUT/c5_copies$c.json 2> $OUT/c5_copies$c.err
done
timeout -k 10 200 python3 -u tools/conc_sweep.py --copies 2 --churn 0,256 --threads 8,16 > $OUT/sweep_copies2.jsonl 2>> $OUT/sweep.err
