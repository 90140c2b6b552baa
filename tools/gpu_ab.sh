#!/bin/bash
# A/B of study builds on the headline bench (timed region only: no latency,
# caller, host-fed, parity or CPU legs), alternating builds ROUNDS times.
# usage: [BENCH_ARGS="--config c3deep"] tools/gpu_ab.sh <tag> <rounds> <variant>...   (emqx_amd/variants/libtmatch_<variant>.so)
set -e
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    TM_LIB=emqx_amd/variants/libtmatch_$v.so timeout -k 10 150 python3 -u bench.py --steps 300 --latency-batches 0 \
      --no-cpu --no-parity $BENCH_ARGS > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('kernel_avg_ms'))" $OUT/${v}_$r.json $v >> $OUT/ab.txt
  done
done
cat $OUT/ab.txt
