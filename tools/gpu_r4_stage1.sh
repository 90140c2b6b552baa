#!/bin/bash
# Round 4 study: small batches on the staged lane walk (tools/study/mk_stage1.py).
set -e
OUT=gpurun_out/stage1_$1
mkdir -p $OUT
TM_LIB=emqx_amd/variants/libtmatch_stage1.so timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q \
  --timeout 200 --timeout-method thread -k "random_sets or golden or wildcard or first or concurrent" > $OUT/tests.log 2>&1 || true
for rep in 1 2; do
  for v in prod stage1; do
    lib=emqx_amd/variants/libtmatch_$v.so; [ $v = prod ] && lib=emqx_amd/libtmatch.so
    TM_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu --no-parity > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err
  done
done
echo done > $OUT/done.txt
