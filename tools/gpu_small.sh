#!/bin/bash
# One-launch small-batch check: the GPU suite's small-batch / parity tests, the
# concurrent-caller sweep (in place and HBM), and a kernel trace of 4k batches.
# usage: tools/gpu_small.sh <tag> [full]
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" = "full" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
else
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "small or wave or random_sets or c1_full or edge or deep or first_batch or hash_not_last or concurrent or zero_copy or staged" > $OUT/gputest.log 2>&1
fi
tail -1 $OUT/gputest.log
timeout -k 10 200 python3 -u tools/conc_sweep.py --churn 0,256 --threads 1,8,16 > $OUT/sweep.jsonl 2>> $OUT/sweep.err
timeout -k 10 200 python3 -u tools/conc_sweep.py --dev 1 --churn 0 --threads 1,8 >> $OUT/sweep.jsonl 2>> $OUT/sweep.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/lat -o run --output-format csv -- \
  python3 -u tools/latency_trace.py --batch 4096 --reps 60 > $OUT/lat.log 2>&1
