#!/bin/bash
# Small-batch change check: GPU parity subset, callers sweep (in place, with and
# without churn; HBM), 4k kernel trace, then the N=2 bench rehearsal on one GPU
# over gloo.  usage: tools/gpu_small2.sh <tag>
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "small or wave or random_sets or c1_full or edge or deep or first_batch or hash_not_last or concurrent or zero_copy or staged or c2 or long_runs or golden or router or broker" > $OUT/gputest.log 2>&1
tail -1 $OUT/gputest.log
timeout -k 10 200 python3 -u tools/conc_sweep.py --churn 0,256 --threads 1,8,16 > $OUT/sweep.jsonl 2>> $OUT/sweep.err
timeout -k 10 200 python3 -u tools/conc_sweep.py --dev 1 --churn 0 --threads 8 >> $OUT/sweep.jsonl 2>> $OUT/sweep.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/lat -o run --output-format csv -- \
  python3 -u tools/latency_trace.py --batch 4096 --reps 60 > $OUT/lat.log 2>&1
