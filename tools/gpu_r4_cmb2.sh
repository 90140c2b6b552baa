#!/bin/bash
# Round 4: combiner leader count (concurrent combined launches) 0 / 2 / 3 / 4 / 6.
set -e
OUT=gpurun_out/cmb_$1
mkdir -p $OUT
for rep in 1 2; do
  for v in nocmb cmb2 prod cmb4 cmb6; do
    lib=emqx_amd/variants/libtmatch_$v.so; [ $v = prod ] && lib=emqx_amd/libtmatch.so
    TM_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu --no-parity --latency-batches 2 \
      > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err
  done
done
echo done > $OUT/done.txt
