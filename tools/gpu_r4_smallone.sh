#!/bin/bash
# Round 4 study: batches <= 64k topics on k_walk_one (lane per topic) instead of k_walk_small.
set -e
OUT=gpurun_out/smallone_$1
mkdir -p $OUT
TM_LIB=emqx_amd/variants/libtmatch_smallone.so timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q \
  --timeout 200 --timeout-method thread -k "random_sets or small or wildcard or golden" > $OUT/tests.log 2>&1
for rep in 1 2; do
  for v in prod smallone; do
    lib=emqx_amd/variants/libtmatch_$v.so; [ $v = prod ] && lib=emqx_amd/libtmatch.so
    TM_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err
  done
done
echo done > $OUT/done.txt
