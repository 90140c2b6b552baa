#!/bin/bash
# C5 at the same delta rate in two cadences: 100 deltas before every step, and
# the router syncer's batch size (1000 deltas every 10 steps), 1 and 3 streams.
# usage: tools/gpu_c5cad.sh <tag>
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
B="--config c5 --no-cpu --latency-batches 0 --concurrency 0"
timeout -k 10 400 python -u bench.py $B > $OUT/c5_100x1.json 2> $OUT/c5_100x1.err
timeout -k 10 400 python -u bench.py $B --deltas 1000 --delta-every 10 --streams 3 > $OUT/c5_1000x10_s3.json 2> $OUT/c5_1000x10_s3.err
timeout -k 10 400 python -u bench.py $B --deltas 1000 --delta-every 10 --streams 1 > $OUT/c5_1000x10_s1.json 2> $OUT/c5_1000x10_s1.err
