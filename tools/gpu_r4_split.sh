#!/bin/bash
# Round 4: sub-batches per step (bench.py --split) at the driver's step count and the default.
set -e
OUT=gpurun_out/split_$1
mkdir -p $OUT
F="--latency-batches 0 --concurrency 0 --no-cpu"
for rep in 1 2; do
  for sp in 1 3 2; do
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --split $sp $F > $OUT/s${sp}_20_$rep.json 2> $OUT/s${sp}_20_$rep.err
  done
done
for sp in 1 3; do
  timeout -k 10 300 python3 -u bench.py --split $sp $F > $OUT/s${sp}_100.json 2> $OUT/s${sp}_100.err
done
echo done > $OUT/done.txt
