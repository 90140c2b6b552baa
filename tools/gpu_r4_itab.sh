#!/bin/bash
# Round 4 study: level-D children stored as node lines in
# their parent's child table (tools/study/mk_itab.py builds the variants).
# Per build x depth set: a short bench line (isolated walk, 20k-topic parity
# sample vs the oracle) and two PMC passes over the profiling driver.
# usage: tools/gpu_r4_itab.sh <tag> "<name>:<lib>:<depths>" ...
set -e
OUT=gpurun_out/itab_$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
for spec in "$@"; do
  IFS=: read name lib dep <<< "$spec"
  echo "== $name $lib depths=$dep" >> $OUT/progress.txt
  TM_LIB=$lib TM_STUDY_ITAB=$dep timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --latency-batches 0 \
    --concurrency 0 --no-cpu > $OUT/$name.json 2> $OUT/$name.err
  i=0
  for pmc in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
    i=$((i+1))
    TM_LIB=$lib TM_STUDY_ITAB=$dep timeout -k 10 -s KILL 120 rocprofv3 --pmc $pmc -d $OUT/${name}_p$i -o run \
      --output-format csv -- python3 -u tools/profile_walk.py --config c3 --batches 8 > $OUT/${name}_p$i.log 2>&1
  done
done
echo done >> $OUT/progress.txt
