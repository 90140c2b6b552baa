#!/bin/bash
# Round 4 study: in-place host batches with their inputs copied by DMA (study build dmain).
set -e
OUT=gpurun_out/dmain_$1
mkdir -p $OUT
for rep in 1 2; do
  for v in prod dmain; do
    lib=emqx_amd/variants/libtmatch_$v.so; [ $v = prod ] && lib=emqx_amd/libtmatch.so
    TM_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err
  done
done
echo done > $OUT/done.txt
