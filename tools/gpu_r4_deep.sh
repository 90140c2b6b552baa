#!/bin/bash
# Round 4: c3deep (10% of topics 33-64 levels) on the two-phase path vs k_walk_one.
set -e
OUT=gpurun_out/deep_$1
mkdir -p $OUT
F="--config c3deep --latency-batches 0 --concurrency 0 --no-cpu"
for rep in 1 2; do
  for p in phases one; do
    timeout -k 10 300 python3 -u bench.py --large-path $p $F > $OUT/${p}_$rep.json 2> $OUT/${p}_$rep.err
  done
done
for d in 0 8 1000000000; do
  timeout -k 10 120 python3 -u tools/profile_walk.py --config c3deep --large-path one --lb-defer $d --streams 1 --batches 16 2>&1 \
    | grep -v amdgpu.ids >> $OUT/walk.txt
done
timeout -k 10 120 python3 -u tools/profile_walk.py --config c3deep --large-path phases --streams 1 --batches 16 2>&1 \
  | grep -v amdgpu.ids >> $OUT/walk.txt
echo done > $OUT/done.txt
