#!/bin/bash
# Divergence study: the isolated C3 walk on batches in generator order vs
# ordered by predicted work (so a wave's lanes walk similar numbers of states).
# usage: tools/gpu_work_order.sh <tag>
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
for o in stream work stream work; do
  timeout -k 10 300 python3 -u tools/profile_walk.py --order $o --batches 16 >> $OUT/timing.txt 2>> $OUT/err.txt
done
