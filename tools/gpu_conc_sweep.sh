#!/bin/bash
# Concurrent-caller sweep over HIP hardware-queue counts (tools/conc_sweep.py),
# then a kernel trace of 8 callers without churn.  usage: tools/gpu_conc_sweep.sh <tag>
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 -u tools/conc_sweep.py >> $OUT/sweep.jsonl 2>> $OUT/sweep.err
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/p8 -o run -- \
  python3 -u tools/callers_trace.py --threads 8 > $OUT/p8.log 2>&1
python3 tools/overlap.py $OUT/p8/run_kernel_trace.csv k_walk_small > $OUT/p8_overlap.txt
