#!/bin/bash
# Study: memory-side requests of the walk with the batch in generator order vs
# byte-sorted vs bucketed by the first two levels (tools/profile_walk.py --order).
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r5_orderpmc
mkdir -p $OUT
for o in stream sorted bucket; do
  timeout -k 10 -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/$o -o run --output-format csv -- \
    python3 -u tools/profile_walk.py --order $o > $OUT/$o.log 2>&1
done
