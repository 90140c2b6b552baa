#!/bin/bash
# Round 4: the host-batch combiner -- its GPU tests, then bench lines with it (product) and without (nocmb).
set -e
OUT=gpurun_out/cmb_$1
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "combined or u32 or concurrent or lookback or broker or router" > $OUT/tests.log 2>&1
for rep in 1 2; do
  for v in prod nocmb; do
    lib=emqx_amd/variants/libtmatch_$v.so; [ $v = prod ] && lib=emqx_amd/libtmatch.so
    TM_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err
  done
done
echo done > $OUT/done.txt
