#!/bin/bash
# Do concurrent callers' kernels overlap?  Kernel traces of 4 native caller
# threads (no churn), product library and the variant without the one-launch path.
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/p4 -o run -- \
  python3 -u tools/callers_trace.py --threads 4 > $OUT/p4.log 2>&1
TM_LIB=emqx_amd/variants/libtmatch_nofused.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
  -d $OUT/n4 -o run -- python3 -u tools/callers_trace.py --threads 4 > $OUT/n4.log 2>&1
timeout -k 10 200 python3 -u tools/callers_trace.py --threads 1 > $OUT/p1.log 2>&1
