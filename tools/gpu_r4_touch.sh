#!/bin/bash
# Round 4 study: touch the '+' child's line during the literal probe (tools/study/mk_touch.py).
set -e
OUT=gpurun_out/touch_$1
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in prod touch2; do
    lib=emqx_amd/variants/libtmatch_$v.so; [ $v = prod ] && lib=emqx_amd/libtmatch.so
    echo "== $v $rep" >> $OUT/walk.txt
    TM_LIB=$lib timeout -k 10 120 python3 -u tools/profile_walk.py --config c3 --large-path phases --streams 1 --batches 24 2>&1 \
      | grep -v amdgpu.ids >> $OUT/walk.txt
  done
done
TM_LIB=emqx_amd/variants/libtmatch_touch2.so timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_touch2 -o run \
  --output-format csv -- python3 -u tools/profile_walk.py --config c3 --batches 8 > $OUT/pmc_touch2.log 2>&1
for v in prod touch2; do
  lib=emqx_amd/variants/libtmatch_$v.so; [ $v = prod ] && lib=emqx_amd/libtmatch.so
  TM_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --latency-batches 0 --concurrency 0 --no-cpu \
    > $OUT/${v}_20.json 2> $OUT/${v}_20.err
done
echo done > $OUT/done.txt
