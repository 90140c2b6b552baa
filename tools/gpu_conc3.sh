#!/bin/bash
# 4k-topic callers with HBM buffers through the device API vs in place in host
# memory (tools/conc_sweep.py), no churn.  usage: tools/gpu_conc3.sh <tag>
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/conc_sweep.py --dev 1 --churn 0 >> $OUT/sweep.jsonl 2>> $OUT/sweep.err
