#!/bin/bash
# Round 4: streams per step at the driver's step count (20 steps, 5 warmup).
set -e
OUT=gpurun_out/streams_$1
mkdir -p $OUT
F="--latency-batches 0 --concurrency 0 --no-cpu --no-parity"
for rep in 1 2; do
  for st in 3 2 4; do
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --streams $st $F > $OUT/st${st}_$rep.json 2> $OUT/st${st}_$rep.err
  done
done
echo done > $OUT/done.txt
