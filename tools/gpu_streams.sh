#!/bin/bash
# Headline bench (timed region only) at several stream counts, alternating.
# usage: tools/gpu_streams.sh <tag> <rounds> <streams>...
set -e
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/streams_$TAG
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for ns in "$@"; do
    timeout -k 10 150 python3 -u bench.py --steps 300 --latency-batches 0 --no-cpu --no-parity --streams $ns \
      > $OUT/s${ns}_$r.json 2> $OUT/s${ns}_$r.err
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('streams', sys.argv[2], d['value'], d['ms_per_step'])" $OUT/s${ns}_$r.json $ns >> $OUT/ab.txt
  done
done
cat $OUT/ab.txt
