#!/bin/bash
# Round 4 study: the short kernels on a high-priority stream (tools/study/mk_prio.py).
set -e
OUT=gpurun_out/prio_$1
mkdir -p $OUT
F="--latency-batches 0 --concurrency 0 --no-cpu"
for rep in 1 2; do
  for v in prod prio fork; do
    lib=emqx_amd/variants/libtmatch_$v.so; [ $v = prod ] && lib=emqx_amd/libtmatch.so
    TM_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 $F > $OUT/${v}_20_$rep.json 2> $OUT/${v}_20_$rep.err
  done
done
for v in prod prio; do
  lib=emqx_amd/variants/libtmatch_$v.so; [ $v = prod ] && lib=emqx_amd/libtmatch.so
  TM_LIB=$lib timeout -k 10 300 python3 -u bench.py $F > $OUT/${v}_100.json 2> $OUT/${v}_100.err
done
echo done > $OUT/done.txt
