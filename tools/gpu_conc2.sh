#!/bin/bash
# Where a concurrent caller's batch time goes: host-side phase timings
# (TM_HOST_TIMING) at 1 and 8 threads, and the stamped study build's per-phase
# device times of a 4k batch.  usage: tools/gpu_conc2.sh <tag>
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
for t in 1 8; do
  TM_HOST_TIMING=1 timeout -k 10 200 python3 -u tools/callers_trace.py --threads $t --seconds 0.3 > $OUT/ht$t.log 2> $OUT/ht$t.err
  python3 tools/host_timing_summary.py $OUT/ht$t.err > $OUT/ht$t.txt
done
TM_LIB=emqx_amd/variants/libtmatch_stamps.so timeout -k 10 250 python3 -u tools/stamps_study.py > $OUT/stamps.log 2>&1
