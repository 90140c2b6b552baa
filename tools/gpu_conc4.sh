#!/bin/bash
# Which PCIe leg of an in-place 4k batch costs what under 8 callers: all HBM
# (dev 1), outputs to host (dev 2), inputs from host (dev 3), all host (dev 0).
# usage: tools/gpu_conc4.sh <tag>
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
for d in 0 1 2 3; do
  timeout -k 10 200 python3 -u tools/conc_sweep.py --dev $d --churn 0 --threads 1,8 >> $OUT/sweep.jsonl 2>> $OUT/sweep.err
done
