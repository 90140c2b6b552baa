#!/bin/bash
# Round 4 study: in-place small batches signal completion through a mapped word (tools/study/mk_spin.py).
set -e
OUT=gpurun_out/spin_$1
mkdir -p $OUT
TM_LIB=emqx_amd/variants/libtmatch_spin.so timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q \
  --timeout 200 --timeout-method thread -k "lookback or u32 or concurrent or random_sets or small or in_place or host or replicas" \
  > $OUT/tests.log 2>&1
for rep in 1 2; do
  for v in prod spin; do
    lib=emqx_amd/variants/libtmatch_$v.so; [ $v = prod ] && lib=emqx_amd/libtmatch.so
    TM_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err
  done
done
echo done > $OUT/done.txt
