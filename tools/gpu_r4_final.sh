#!/bin/bash
# Round 4 final tree: the default bench line, the driver-shaped line, the
# replica-topology rehearsal (2 replicas on this one GPU).
set -e
OUT=gpurun_out/r4_final
mkdir -p $OUT
timeout -k 10 400 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $OUT/bench_20.json 2> $OUT/bench_20.err
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --latency-batches 0 --concurrency 0 --no-cpu --replicas 2 \
  > $OUT/bench_rep2.json 2> $OUT/bench_rep2.err
echo done > $OUT/done.txt
